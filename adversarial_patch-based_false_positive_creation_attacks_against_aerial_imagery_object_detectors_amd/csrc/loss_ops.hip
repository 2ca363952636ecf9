// Loss head: per-anchor objectness/class extraction at the patch cell and the
// creation-attack losses (reference train_patch.py:428-548, 230-253), forward
// and the sparse gradient into the head tensors.  One workgroup; one thread per
// image; the batch means are summed by thread 0 in image order (deterministic).
#pragma clang fp contract(off)
#include "common.h"
#include <math.h>

namespace {
constexpr int MAXH = 4;          // heads
constexpr int NCLS = 15;         // train_patch.py:459 hard-codes 5+15 channels per anchor
constexpr int NF = 5 + NCLS;
constexpr int MAXB = 4096;

struct LossArgs {
  const float* heads[MAXH];
  float* dheads[MAXH];
  int hw[MAXH];
  int nheads, Cp, B, S, target, objective;
  const float* g2;
};

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

// torch.div(a, b, rounding_mode='floor') for float32 (ATen div_floor)
__device__ __forceinline__ float div_floor(float a, float b) {
  float mod = fmodf(a, b);
  float div = (a - mod) / b;
  if (mod != 0.f && ((b < 0.f) != (mod < 0.f))) div -= 1.f;
  float fl;
  if (div != 0.f) {
    fl = floorf(div);
    if (div - fl > 0.5f) fl += 1.f;
  } else {
    fl = copysignf(0.f, a / b);
  }
  return fl;
}

__global__ __launch_bounds__(256) void cell_loss_k(LossArgs a, const float* __restrict__ center,
                                                   float* __restrict__ out2, float* __restrict__ obj_out,
                                                   float* __restrict__ cls_out, int32_t* __restrict__ cells,
                                                   int32_t* __restrict__ flags) {
  __shared__ float s_max[MAXB];
  __shared__ float s_cls[MAXB];
  __shared__ int s_flag;
  if (threadIdx.x == 0) s_flag = 0;
  __syncthreads();
  const int A = 3 * a.nheads;
  const float invB = 1.f / (float)a.B;
  const float g_obj = a.g2 ? a.g2[0] : 0.f, g_cls = a.g2 ? a.g2[1] : 0.f;
  for (int b = threadIdx.x; b < a.B; b += blockDim.x) {
    float obj[3 * MAXH];
    int idx[MAXH];
    float best = 0.f;
    int kbest = -1;
    float cls_term = 0.f;
    for (int h = 0; h < a.nheads; ++h) {
      const int hw = a.hw[h];
      const float stride = (float)((double)a.S / (double)hw);       // train_patch.py:446
      const int ix = (int)div_floor(center[2 * b + 0], stride);     // 449-450, 463
      const int iy = (int)div_floor(center[2 * b + 1], stride);     // 464
      int index = ix * hw + iy;                                      // 467
      if (index < 0 || index >= hw * hw) {
        atomicOr(&s_flag, 1);
        index = index < 0 ? 0 : hw * hw - 1;
      }
      idx[h] = index;
      if (cells) cells[h * a.B + b] = index;
      const float* cell = a.heads[h] + ((size_t)b * hw * hw + index) * a.Cp;
      for (int an = 0; an < 3; ++an) {
        const int k = h * 3 + an;
        const float* f = cell + an * NF;
        const float o = sigm(f[4]);                                  // 470-476
        obj[k] = o;
        if (obj_out) obj_out[(size_t)b * A + k] = o;
        if (kbest < 0 || o > best) { best = o; kbest = k; }          // torch.max: first index
        float p[NCLS];
        float mx = -INFINITY;
        int cmax = 0;
        for (int c = 0; c < NCLS; ++c) {
          p[c] = sigm(f[5 + c]);                                     // 481
          if (cls_out) cls_out[((size_t)b * A + k) * NCLS + c] = p[c];
          if (p[c] > mx) { mx = p[c]; cmax = c; }
        }
        float* dcell = a.dheads[h] ? a.dheads[h] + ((size_t)b * hw * hw + index) * a.Cp + an * NF : nullptr;
        if (a.objective == 0) {
          // CrossEntropyLoss on probabilities (train_patch.py:534-546)
          float se = 0.f;
          for (int c = 0; c < NCLS; ++c) se += expf(p[c] - mx);
          const float lse = mx + logf(se);
          cls_term += lse - p[a.target];
          if (dcell) {
            const float g = g_cls * invB / (float)A;
            for (int c = 0; c < NCLS; ++c) {
              float sm = expf(p[c] - mx) / se;
              float dp = g * (sm - (c == a.target ? 1.f : 0.f));
              dcell[5 + c] = dp * p[c] * (1.f - p[c]);
            }
          }
        } else if (a.objective == 1) {
          // noCLS_loss_targeted (train_patch.py:565-575): sum_b mean_k (max - target)
          cls_term += mx - p[a.target];
          if (dcell) {
            const float g = g_cls / (float)A;
            for (int c = 0; c < NCLS; ++c) {
              float dp = (c == cmax ? g : 0.f) - (c == a.target ? g : 0.f);
              dcell[5 + c] = dp * p[c] * (1.f - p[c]);
            }
          }
        } else if (dcell) {
          for (int c = 0; c < NCLS; ++c) dcell[5 + c] = 0.f;
        }
        if (dcell) dcell[4] = 0.f;
      }
    }
    s_max[b] = best;
    s_cls[b] = cls_term / (a.objective == 0 ? (float)A : (a.objective == 1 ? (float)A : 1.f));
    // objectness gradient: d/d obj[kbest] of 4*(1 - mean_b max_k obj) = -4/B
    const int h = kbest / 3, an = kbest % 3;
    if (a.dheads[h]) {
      float* dcell = a.dheads[h] + ((size_t)b * a.hw[h] * a.hw[h] + idx[h]) * a.Cp + an * NF;
      const float o = obj[kbest];
      dcell[4] = (-4.f * invB * g_obj) * o * (1.f - o);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float sm = 0.f, sc = 0.f;
    for (int b = 0; b < a.B; ++b) {
      sm += s_max[b];
      sc += s_cls[b];
    }
    out2[0] = 4.f * (1.f - sm / (float)a.B);                       // train_patch.py:236-239
    out2[1] = a.objective == 0 ? sc / (float)a.B : (a.objective == 1 ? sc : 0.f);
    if (flags) flags[0] = s_flag;
  }
}
}  // namespace

extern "C" int po_cell_loss(const float* const* heads, const int* hw, int nheads, int Cp, int B, int S,
                            const float* center, int target, int objective, const float* g2,
                            float* const* d_heads, float* out2, float* obj_out, float* cls_out,
                            int32_t* cells, int32_t* flags, po_stream_t s) {
  PO_REQUIRE(heads && hw && center && out2, "po_cell_loss: null pointer");
  PO_REQUIRE(nheads >= 1 && nheads <= MAXH, "po_cell_loss: 1..%d heads supported, got %d", MAXH, nheads);
  PO_REQUIRE(Cp >= 3 * NF, "po_cell_loss: head channel stride %d < 60 (3 anchors x (5+15))", Cp);
  PO_REQUIRE(B >= 1 && B <= MAXB, "po_cell_loss: batch %d out of range", B);
  PO_REQUIRE(target >= 0 && target < NCLS, "po_cell_loss: target %d out of range", target);
  PO_REQUIRE(objective >= 0 && objective <= 2, "po_cell_loss: objective must be 0,1,2");
  PO_REQUIRE(!d_heads || g2, "po_cell_loss: g2 required with d_heads");
  LossArgs a;
  for (int h = 0; h < MAXH; ++h) {
    a.heads[h] = h < nheads ? heads[h] : nullptr;
    a.dheads[h] = (d_heads && h < nheads) ? d_heads[h] : nullptr;
    a.hw[h] = h < nheads ? hw[h] : 1;
    if (h < nheads) PO_REQUIRE(heads[h] && hw[h] > 0, "po_cell_loss: bad head %d", h);
  }
  a.nheads = nheads;
  a.Cp = Cp;
  a.B = B;
  a.S = S;
  a.target = target;
  a.objective = objective;
  a.g2 = g2;
  hipLaunchKernelGGL(cell_loss_k, dim3(1), dim3(256), 0, po::stream_of(s), a, center, out2, obj_out,
                     cls_out, cells, flags);
  return po::check_launch("po_cell_loss");
}
