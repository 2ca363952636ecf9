// Loss head: per-anchor objectness/class extraction at the patch cell and the
// creation-attack losses (reference train_patch.py:428-548, 230-253), forward
// and the sparse gradient into the head tensors.  One thread per (image,
// anchor), per-image reductions in anchor order, and the batch means summed by
// one thread in image order (deterministic); chunks of 16 images run on one
// workgroup each when the caller gives a scratch buffer.
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
  const int32_t* org[MAXH];   // window origin [B,2] or NULL (full map)
  int hw[MAXH], win[MAXH];    // map side, stored side
  int nheads, Cp, B, S, target, objective;
  const float* g2;
};

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

// One thread per (image, anchor) of a chunk of CL_IMG images (the anchors'
// sigmoid / class / CE work runs in parallel); then one thread per image of
// the chunk takes the first-index max objectness and sums the class terms in
// anchor order, as the one-thread-per-image form did (same values, same order).
constexpr int CL_IMG = 16;
// With a scratch buffer the chunks are spread over workgroups (one per chunk)
// and each image's (max objectness, class term) goes to scratch[b],
// scratch[B + b]; cell_final_k then sums them in image order, so the result
// is bit-identical to the one-workgroup form.
__global__ __launch_bounds__(256) void cell_loss_k(LossArgs a, const float* __restrict__ center,
                                                   float* __restrict__ out2, float* __restrict__ obj_out,
                                                   float* __restrict__ cls_out, int32_t* __restrict__ cells,
                                                   int32_t* __restrict__ flags, float* __restrict__ scratch) {
  __shared__ float s_max[MAXB];
  __shared__ float s_cls[MAXB];
  __shared__ float c_obj[CL_IMG][3 * MAXH];
  __shared__ float c_cls[CL_IMG][3 * MAXH];
  __shared__ int c_off[CL_IMG][MAXH];
  __shared__ int s_flag;
  if (threadIdx.x == 0) s_flag = 0;
  __syncthreads();
  const int A = 3 * a.nheads;
  const float invB = 1.f / (float)a.B;
  const float g_obj = a.g2 ? a.g2[0] : 0.f, g_cls = a.g2 ? a.g2[1] : 0.f;
  for (int b0 = blockIdx.x * CL_IMG; b0 < a.B; b0 += gridDim.x * CL_IMG) {
    const int lb = threadIdx.x / A, k = threadIdx.x - lb * A;
    const int b = b0 + lb;
    if (lb < CL_IMG && b < a.B) {
      const int h = k / 3, an = k - h * 3;
      const int hw = a.hw[h];
      bool oob;
      const int index = po::head_cell(center[2 * b + 0], center[2 * b + 1], a.S, hw, &oob);
      if (oob) atomicOr(&s_flag, 1);
      if (cells && an == 0) cells[h * a.B + b] = index;
      int r = index / hw, c = index - (index / hw) * hw;
      if (a.org[h]) {
        r -= a.org[h][2 * b];
        c -= a.org[h][2 * b + 1];
        if (r < 0 || r >= a.win[h] || c < 0 || c >= a.win[h]) {
          atomicOr(&s_flag, 2);
          r = min(max(r, 0), a.win[h] - 1);
          c = min(max(c, 0), a.win[h] - 1);
        }
      }
      const size_t off = (((size_t)b * a.win[h] + r) * a.win[h] + c) * a.Cp;
      if (an == 0) c_off[lb][h] = (int)(off / a.Cp);
      const float* f = a.heads[h] + off + an * NF;
      const float o = sigm(f[4]);                                    // 470-476
      c_obj[lb][k] = o;
      if (obj_out) obj_out[(size_t)b * A + k] = o;
      float p[NCLS];
      float mx = -INFINITY;
      int cmax = 0;
      for (int cc = 0; cc < NCLS; ++cc) {
        p[cc] = sigm(f[5 + cc]);                                     // 481
        if (cls_out) cls_out[((size_t)b * A + k) * NCLS + cc] = p[cc];
        if (p[cc] > mx) { mx = p[cc]; cmax = cc; }
      }
      float* dcell = a.dheads[h] ? a.dheads[h] + off + an * NF : nullptr;
      float cls_term = 0.f;
      if (a.objective == 0) {
        // CrossEntropyLoss on probabilities (train_patch.py:534-546)
        float se = 0.f;
        for (int cc = 0; cc < NCLS; ++cc) se += expf(p[cc] - mx);
        const float lse = mx + logf(se);
        cls_term = lse - p[a.target];
        if (dcell) {
          const float g = g_cls * invB / (float)A;
          for (int cc = 0; cc < NCLS; ++cc) {
            float sm = expf(p[cc] - mx) / se;
            float dp = g * (sm - (cc == a.target ? 1.f : 0.f));
            dcell[5 + cc] = dp * p[cc] * (1.f - p[cc]);
          }
        }
      } else if (a.objective == 1) {
        // noCLS_loss_targeted (train_patch.py:565-575): sum_b mean_k (max - target)
        cls_term = mx - p[a.target];
        if (dcell) {
          const float g = g_cls / (float)A;
          for (int cc = 0; cc < NCLS; ++cc) {
            float dp = (cc == cmax ? g : 0.f) - (cc == a.target ? g : 0.f);
            dcell[5 + cc] = dp * p[cc] * (1.f - p[cc]);
          }
        }
      } else if (dcell) {
        for (int cc = 0; cc < NCLS; ++cc) dcell[5 + cc] = 0.f;
      }
      if (dcell) dcell[4] = 0.f;
      c_cls[lb][k] = cls_term;
    }
    __syncthreads();
    const int fb = b0 + (int)threadIdx.x;
    if ((int)threadIdx.x < CL_IMG && fb < a.B) {
      const int lb2 = threadIdx.x;
      float best = 0.f, cls_term = 0.f;
      int kbest = -1;
      for (int kk = 0; kk < A; ++kk) {
        const float o = c_obj[lb2][kk];
        if (kbest < 0 || o > best) { best = o; kbest = kk; }          // torch.max: first index
        cls_term += c_cls[lb2][kk];
      }
      const float ct = cls_term / (a.objective == 0 ? (float)A : (a.objective == 1 ? (float)A : 1.f));
      if (scratch) {
        scratch[fb] = best;
        scratch[a.B + fb] = ct;
      } else {
        s_max[fb] = best;
        s_cls[fb] = ct;
      }
      // objectness gradient: d/d obj[kbest] of 4*(1 - mean_b max_k obj) = -4/B
      const int h = kbest / 3, an = kbest % 3;
      if (a.dheads[h]) {
        float* dcell = a.dheads[h] + (size_t)c_off[lb2][h] * a.Cp + an * NF;
        dcell[4] = (-4.f * invB * g_obj) * best * (1.f - best);
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (!scratch) {
      float sm = 0.f, sc = 0.f;
      for (int b = 0; b < a.B; ++b) {
        sm += s_max[b];
        sc += s_cls[b];
      }
      out2[0] = 4.f * (1.f - sm / (float)a.B);                       // train_patch.py:236-239
      out2[1] = a.objective == 0 ? sc / (float)a.B : (a.objective == 1 ? sc : 0.f);
    }
    if (flags && s_flag) atomicOr(flags, s_flag);       // accumulates over calls
  }
}

// batch means of the per-image terms, summed in image order (as cell_loss_k's one-workgroup form)
__global__ __launch_bounds__(256) void cell_final_k(const float* __restrict__ scratch, int B, int objective,
                                                    float* __restrict__ out2) {
  __shared__ float s_max[MAXB];
  __shared__ float s_cls[MAXB];
  for (int b = threadIdx.x; b < B; b += 256) {
    s_max[b] = scratch[b];
    s_cls[b] = scratch[B + b];
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  float sm = 0.f, sc = 0.f;
  for (int b = 0; b < B; ++b) {
    sm += s_max[b];
    sc += s_cls[b];
  }
  out2[0] = 4.f * (1.f - sm / (float)B);                           // train_patch.py:236-239
  out2[1] = objective == 0 ? sc / (float)B : (objective == 1 ? sc : 0.f);
}
}  // namespace

extern "C" int po_cell_loss(const float* const* heads, const int* hw, const int* win,
                            const int32_t* const* org, int nheads, int Cp, int B, int S,
                            const float* center, int target, int objective, const float* g2,
                            float* const* d_heads, float* out2, float* obj_out, float* cls_out,
                            int32_t* cells, int32_t* flags, float* scratch, po_stream_t s) {
  PO_REQUIRE(heads && hw && center && out2, "po_cell_loss: null pointer");
  PO_REQUIRE(nheads >= 1 && nheads <= MAXH, "po_cell_loss: 1..%d heads supported, got %d", MAXH, nheads);
  PO_REQUIRE(Cp >= 3 * NF, "po_cell_loss: head channel stride %d < 60 (3 anchors x (5+15))", Cp);
  PO_REQUIRE(B >= 1 && B <= MAXB, "po_cell_loss: batch %d out of range", B);
  PO_REQUIRE(target >= 0 && target < NCLS, "po_cell_loss: target %d out of range", target);
  PO_REQUIRE(objective >= 0 && objective <= 2, "po_cell_loss: objective must be 0,1,2");
  PO_REQUIRE(!d_heads || g2, "po_cell_loss: g2 required with d_heads");
  LossArgs a;
  for (int h = 0; h < MAXH; ++h) {
    const bool on = h < nheads;
    a.heads[h] = on ? heads[h] : nullptr;
    a.dheads[h] = (d_heads && on) ? d_heads[h] : nullptr;
    a.hw[h] = on ? hw[h] : 1;
    a.org[h] = (org && on) ? org[h] : nullptr;
    a.win[h] = a.org[h] ? (win ? win[h] : 0) : a.hw[h];
    if (on) {
      PO_REQUIRE(heads[h] && hw[h] > 0, "po_cell_loss: bad head %d", h);
      PO_REQUIRE(a.win[h] > 0 && a.win[h] <= hw[h], "po_cell_loss: head %d window side %d (map %d)", h,
                 a.win[h], hw[h]);
    }
  }
  a.nheads = nheads;
  a.Cp = Cp;
  a.B = B;
  a.S = S;
  a.target = target;
  a.objective = objective;
  a.g2 = g2;
  const int nchunk = scratch ? po::ceil_div(B, CL_IMG) : 1;
  hipLaunchKernelGGL(cell_loss_k, dim3(nchunk), dim3(256), 0, po::stream_of(s), a, center, out2, obj_out,
                     cls_out, cells, flags, scratch);
  if (scratch)
    hipLaunchKernelGGL(cell_final_k, dim3(1), dim3(256), 0, po::stream_of(s), scratch, B, objective, out2);
  return po::check_launch("po_cell_loss");
}

// ---------------------------------------------------------------------------
// The loss of one iteration from the cell-loss pair and the regularisers
// (train_patch.py:230-314, train_patch.combine_terms), and its gradient: the
// same fp32 operations in the same order as the PyTorch expression and its
// autograd (maximum's backward splits a tie in half), one thread.
namespace {
constexpr float NPS_F = 0.01f, TV_F = 2.5f, TV_FLOOR = 0.1f;
__global__ void loss_combine_k(const float* __restrict__ out2, const float* __restrict__ reg, float w_img,
                               float w_cls, float w_patch, int weighted, int with_cls, float* __restrict__ terms,
                               float* __restrict__ loss_out) {
  float no_obj = out2[0], no_cls = out2[1];
  float nps_loss = reg[0] * NPS_F, tv_loss = reg[1] * TV_F, colorful = reg[2];
  float tv_term = fmaxf(tv_loss, TV_FLOOR);
  if (isnan(tv_loss)) tv_term = tv_loss;                    // torch.maximum propagates NaN
  if (weighted) {
    no_obj *= w_img;
    no_cls *= w_cls;
    nps_loss *= w_patch;
    tv_loss *= w_patch;
    tv_term *= w_patch;
    colorful *= w_patch;
  }
  float loss = nps_loss + tv_term;
  loss = loss + no_obj;
  loss = loss + colorful;
  if (with_cls) loss = loss + no_cls;
  terms[0] = loss;
  terms[1] = nps_loss;
  terms[2] = tv_loss;
  terms[3] = no_obj;
  terms[4] = no_cls;
  terms[5] = colorful;
  if (loss_out) *loss_out = loss;
}

__global__ void loss_combine_bwd_k(const float* __restrict__ reg, const float* __restrict__ g_loss, float w_img,
                                   float w_cls, float w_patch, int weighted, int with_cls, float* __restrict__ d_out2,
                                   float* __restrict__ d_reg) {
  const float g = g_loss[0];
  const float tv_loss = reg[1] * TV_F;
  // tv_term = maximum(tv_loss, 0.1): grad where tv_loss > 0.1, grad / 2 on a tie, 0 below
  const float gt = weighted ? g * w_patch : g;
  const float gtv = tv_loss == TV_FLOOR ? gt / 2.f : (tv_loss < TV_FLOOR ? 0.f : gt);
  d_out2[0] = weighted ? g * w_img : g;
  d_out2[1] = with_cls ? (weighted ? g * w_cls : g) : 0.f;
  d_reg[0] = (weighted ? g * w_patch : g) * NPS_F;
  d_reg[1] = gtv * TV_F;
  d_reg[2] = weighted ? g * w_patch : g;
}
}  // namespace

extern "C" int po_loss_combine(const float* out2, const float* reg, float w_img, float w_cls, float w_patch,
                               int weighted, int with_cls, float* terms, float* loss_out, po_stream_t s) {
  PO_REQUIRE(out2 && reg && terms, "po_loss_combine: null pointer");
  hipLaunchKernelGGL(loss_combine_k, dim3(1), dim3(1), 0, po::stream_of(s), out2, reg, w_img, w_cls, w_patch,
                     weighted, with_cls, terms, loss_out);
  return po::check_launch("po_loss_combine");
}

extern "C" int po_loss_combine_bwd(const float* reg, const float* g_loss, float w_img, float w_cls, float w_patch,
                                   int weighted, int with_cls, float* d_out2, float* d_reg, po_stream_t s) {
  PO_REQUIRE(reg && g_loss && d_out2 && d_reg, "po_loss_combine_bwd: null pointer");
  hipLaunchKernelGGL(loss_combine_bwd_k, dim3(1), dim3(1), 0, po::stream_of(s), reg, g_loss, w_img, w_cls, w_patch,
                     weighted, with_cls, d_out2, d_reg);
  return po::check_launch("po_loss_combine_bwd");
}

// ---------------------------------------------------------------------------
// Receptive-field windows: one thread per (window, image).
namespace {
struct WinArgs {
  int hw[MAXH];
  int nheads, nwin, maxhw, B, S;
};

__global__ __launch_bounds__(256) void cell_windows_k(WinArgs a, const float* __restrict__ center,
                                                      const int32_t* __restrict__ lut,
                                                      const int32_t* __restrict__ ext,
                                                      int32_t* __restrict__ org, int32_t* __restrict__ flags) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= a.nwin * a.B) return;
  const int w = t / a.B, b = t - w * a.B;
  int lo_r = 1 << 30, hi_r = -(1 << 30), lo_c = 1 << 30, hi_c = -(1 << 30);
  for (int h = 0; h < a.nheads; ++h) {
    bool oob;
    const int index = po::head_cell(center[2 * b + 0], center[2 * b + 1], a.S, a.hw[h], &oob);
    const int r = index / a.hw[h], c = index - r * a.hw[h];
    const int32_t* e = lut + ((size_t)(w * a.nheads + h) * a.maxhw) * 2;
    if (e[2 * r] <= e[2 * r + 1]) {
      lo_r = min(lo_r, e[2 * r]);
      hi_r = max(hi_r, e[2 * r + 1]);
    }
    if (e[2 * c] <= e[2 * c + 1]) {
      lo_c = min(lo_c, e[2 * c]);
      hi_c = max(hi_c, e[2 * c + 1]);
    }
  }
  const int side = ext[2 * w], map = ext[2 * w + 1];
  if (lo_r > hi_r) { lo_r = 0; hi_r = 0; }
  if (lo_c > hi_c) { lo_c = 0; hi_c = 0; }
  if (flags && (hi_r - lo_r + 1 > side || hi_c - lo_c + 1 > side)) atomicOr(flags, 4);
  org[2 * t] = min(max(lo_r, 0), map - side);
  org[2 * t + 1] = min(max(lo_c, 0), map - side);
}
}  // namespace

extern "C" int po_cell_windows(const float* center, int B, int S, int nheads, const int* hw, int nwin,
                               const int32_t* lut, int maxhw, const int32_t* ext, int32_t* org,
                               int32_t* flags, po_stream_t s) {
  PO_REQUIRE(center && hw && lut && ext && org, "po_cell_windows: null pointer");
  PO_REQUIRE(nheads >= 1 && nheads <= MAXH && nwin >= 1 && B >= 1, "po_cell_windows: bad sizes");
  WinArgs a;
  for (int h = 0; h < MAXH; ++h) {
    a.hw[h] = h < nheads ? hw[h] : 1;
    if (h < nheads) PO_REQUIRE(hw[h] >= 1 && hw[h] <= maxhw, "po_cell_windows: head %d side %d > maxhw %d", h,
                               hw[h], maxhw);
  }
  a.nheads = nheads;
  a.nwin = nwin;
  a.maxhw = maxhw;
  a.B = B;
  a.S = S;
  hipLaunchKernelGGL(cell_windows_k, dim3(po::ceil_div((int64_t)nwin * B, 256)), dim3(256), 0,
                     po::stream_of(s), a, center, lut, ext, org, flags);
  return po::check_launch("po_cell_windows");
}

// ---------------------------------------------------------------------------
// MaxProbExtractor (load_data.py:125-311): per image, the max over every head,
// anchor and cell of the objectness (field 4) and of the class-cls_id
// confidence (field 5+cls_id), raw or after sigmoid.  bbox_decode
// (load_data.py:63-122) rewrites only fields 0..3, so the maxima read the head
// logits directly.  Flat index of the reference's output_cat [B,5+C,sum 3hw]:
// head offset + a*h*w + (row*w + col) (load_data.py:188-198).
// Grid (B, 2): blockIdx.y = 0 objectness, 1 class.  Each lane scans indices in
// increasing order (strict > keeps the first), then wave shuffles and one LDS
// pass merge (value, index) pairs with torch.max's rules: NaN wins, ties go to
// the smaller index.
namespace {
struct MaxProbArgs {
  const float* heads[MAXH];
  float* dheads[MAXH];       // backward only
  int64_t sb[MAXH];         // element strides: image, channel, pixel
  int64_t sc[MAXH];
  int64_t sp[MAXH];
  int hw[MAXH];              // pixels per map (h*w)
  int base[MAXH];            // flat index offset of the head
  int nheads, nf, field_obj, field_cls, sigmoid_mode;
};

__device__ __forceinline__ bool mp_better(float v, int i, float bv, int bi) {
  const bool vn = v != v, bn = bv != bv;
  if (vn || bn) return vn && (!bn || i < bi);
  return v > bv || (v == bv && i < bi);
}

__global__ __launch_bounds__(256) void max_prob_k(MaxProbArgs a, float* __restrict__ out, int32_t* __restrict__ idx,
                                                  int B) {
  const int b = blockIdx.x, q = blockIdx.y;
  const int field = q == 0 ? a.field_obj : a.field_cls;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int h = 0; h < a.nheads; ++h) {
    const float* base = a.heads[h] + (int64_t)b * a.sb[h];
    const int hw = a.hw[h];
    for (int an = 0; an < 3; ++an) {
      const float* ch = base + (int64_t)(an * a.nf + field) * a.sc[h];
      for (int p = threadIdx.x; p < hw; p += 256) {
        float v = ch[(int64_t)p * a.sp[h]];
        if (a.sigmoid_mode) v = sigm(v);
        const int i = a.base[h] + an * hw + p;
        if (mp_better(v, i, best, bi)) { best = v; bi = i; }
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o);
    const int oi = __shfl_xor(bi, o);
    if (mp_better(ov, oi, best, bi)) { best = ov; bi = oi; }
  }
  __shared__ float s_v[4];
  __shared__ int s_i[4];
  if ((threadIdx.x & 63) == 0) { s_v[threadIdx.x >> 6] = best; s_i[threadIdx.x >> 6] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w)
      if (mp_better(s_v[w], s_i[w], best, bi)) { best = s_v[w]; bi = s_i[w]; }
    out[q * B + b] = best;
    idx[q * B + b] = bi;
  }
}

// backward: one thread per (image, quantity) adds g * d(value)/d(logit) at the
// selected element (objectness and class fields never coincide)
__global__ __launch_bounds__(64) void max_prob_bwd_k(MaxProbArgs a, const int32_t* __restrict__ idx,
                                                     const float* __restrict__ g, int B) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  if (t >= 2 * B) return;
  const int q = t / B, b = t - q * B;
  const int i = idx[t];
  int h = 0;
  while (h + 1 < a.nheads && i >= a.base[h + 1]) ++h;
  const int loc = i - a.base[h], an = loc / a.hw[h], p = loc - an * a.hw[h];
  const int64_t off = (int64_t)b * a.sb[h] + (int64_t)(an * a.nf + (q == 0 ? a.field_obj : a.field_cls)) * a.sc[h] +
                      (int64_t)p * a.sp[h];
  float d = g[t];
  if (a.sigmoid_mode) {
    const float s = sigm(a.heads[h][off]);
    d *= s * (1.f - s);
  }
  a.dheads[h][off] += d;
}

int max_prob_args(MaxProbArgs& a, const float* const* heads, const int* h, const int* w, const int64_t* strides,
                  int nheads, int num_cls, int cls_id, int sigmoid_mode) {
  PO_REQUIRE(heads && h && w && strides, "po_max_prob: null pointer");
  PO_REQUIRE(nheads >= 1 && nheads <= MAXH, "po_max_prob: 1..%d heads supported, got %d", MAXH, nheads);
  PO_REQUIRE(num_cls >= 1 && cls_id >= 0 && cls_id < num_cls, "po_max_prob: cls_id %d of %d classes", cls_id,
             num_cls);
  int64_t base = 0;
  for (int k = 0; k < MAXH; ++k) {
    const bool on = k < nheads;
    a.heads[k] = on ? heads[k] : nullptr;
    a.dheads[k] = nullptr;
    a.sb[k] = on ? strides[3 * k] : 0;
    a.sc[k] = on ? strides[3 * k + 1] : 0;
    a.sp[k] = on ? strides[3 * k + 2] : 0;
    a.hw[k] = on ? h[k] * w[k] : 1;
    a.base[k] = (int)base;
    if (on) {
      PO_REQUIRE(heads[k] && h[k] > 0 && w[k] > 0, "po_max_prob: bad head %d", k);
      base += 3LL * h[k] * w[k];
    }
  }
  PO_REQUIRE(base < (1LL << 31), "po_max_prob: %lld anchors overflow the int32 index", (long long)base);
  a.nheads = nheads;
  a.nf = 5 + num_cls;
  a.field_obj = 4;
  a.field_cls = 5 + cls_id;
  a.sigmoid_mode = sigmoid_mode ? 1 : 0;
  return PO_OK;
}
}  // namespace

extern "C" int po_max_prob(const float* const* heads, const int* h, const int* w, const int64_t* strides, int nheads,
                           int B, int num_cls, int cls_id, int sigmoid_mode, float* out, int32_t* idx, po_stream_t s) {
  MaxProbArgs a;
  if (int rc = max_prob_args(a, heads, h, w, strides, nheads, num_cls, cls_id, sigmoid_mode)) return rc;
  PO_REQUIRE(out && idx && B >= 1 && B <= 65535, "po_max_prob: bad output or batch %d", B);
  hipLaunchKernelGGL(max_prob_k, dim3(B, 2), dim3(256), 0, po::stream_of(s), a, out, idx, B);
  return po::check_launch("po_max_prob");
}

extern "C" int po_max_prob_bwd(const float* const* heads, const int* h, const int* w, const int64_t* strides,
                               int nheads, int B, int num_cls, int cls_id, int sigmoid_mode, const int32_t* idx,
                               const float* g, float* const* d_heads, po_stream_t s) {
  MaxProbArgs a;
  if (int rc = max_prob_args(a, heads, h, w, strides, nheads, num_cls, cls_id, sigmoid_mode)) return rc;
  PO_REQUIRE(idx && g && d_heads && B >= 1, "po_max_prob_bwd: null pointer");
  for (int k = 0; k < nheads; ++k) {
    PO_REQUIRE(d_heads[k], "po_max_prob_bwd: null gradient of head %d", k);
    a.dheads[k] = d_heads[k];          // the pointer table travels by value in the kernel arguments
  }
  hipLaunchKernelGGL(max_prob_bwd_k, dim3(po::ceil_div(2 * B, 64)), dim3(64), 0, po::stream_of(s), a, idx, g, B);
  return po::check_launch("po_max_prob_bwd");
}

// ---------------------------------------------------------------------------
// Gradient cones: one thread per image walks the block program in order.
namespace {
// floor division; the strides on the cone program are 1 or 2 (shift paths)
__device__ __forceinline__ int fdiv(int a, int b) {
  if (b == 1) return a;
  if (b == 2) return a >> 1;                      // arithmetic shift = floor(a / 2)
  return a >= 0 ? a / b : -((-a + b - 1) / b);
}
__device__ __forceinline__ int cdiv(int a, int b) { return -fdiv(-a, b); }

// inclusive source interval [a, b] -> inclusive interval of the destination
// pixels that read a source pixel in it
__device__ __forceinline__ void cone_map(int kind, int k, int s, int pad, int a, int b, int& lo, int& hi) {
  switch (kind) {
    case 0: lo = cdiv(a + pad - k + 1, s); hi = fdiv(b + pad, s); break;   // out o reads [o*s - pad, o*s - pad + k)
    case 2: lo = fdiv(a, 2); hi = fdiv(b, 2); break;
    case 3: lo = a - 1; hi = b; break;
    case 4: lo = 2 * a; hi = 2 * b + 1; break;
    default: lo = a; hi = b; break;
  }
}

// One workgroup per image: the program and the image's boxes are staged in
// LDS, lanes 0 and 1 walk the (dependent) rows there, one axis each, and the
// workgroup writes the boxes back; global-memory latency is paid once per
// box, not once per row.
__global__ __launch_bounds__(64) void grad_boxes_k(const int32_t* __restrict__ roi, int B, int S,
                                                   const int32_t* __restrict__ prog, int nprog, int nbox,
                                                   int32_t* __restrict__ boxes) {
  extern __shared__ int4 sm[];
  int4* sbox = sm;                                    // [nbox]
  int32_t* sprog = reinterpret_cast<int32_t*>(sm + nbox);   // [nprog][8]
  const int b = blockIdx.x;
  for (int k = threadIdx.x; k < nbox; k += 64) sbox[k] = reinterpret_cast<const int4*>(boxes)[(size_t)k * B + b];
  for (int k = threadIdx.x; k < 8 * nprog; k += 64) sprog[k] = prog[k];
  __syncthreads();
  if (threadIdx.x < 2) {
    // lane 0 walks the row intervals, lane 1 the column intervals (a box's
    // two axes are set together; "skip this row" is agreed by a lane swap)
    const int d = threadIdx.x;
    int* sb = reinterpret_cast<int*>(sbox);            // box k: [r0, c0, r1, c1] at 4 k
    for (int r = 0; r < nprog; ++r) {
      sb[4 * sprog[8 * r] + d] = 0;
      sb[4 * sprog[8 * r] + d + 2] = 0;
    }
    for (int r = 0; r < nprog; ++r) {
      const int32_t* p = sprog + 8 * r;
      int s0, s1;                                      // source interval, half-open
      if (p[1] < 0) {
        if (roi) { s0 = roi[4 * b + 1 - d]; s1 = roi[4 * b + 3 - d]; }   // roi = x0, y0, x1, y1
        else { s0 = 0; s1 = S; }
      } else {
        s0 = sb[4 * p[1] + d];
        s1 = sb[4 * p[1] + d + 2];
      }
      int bad = s0 >= s1;
      bad |= __shfl_xor(bad, 1);
      if (bad) continue;
      int lo, hi;
      cone_map(p[2], p[3], p[4], p[5], s0, s1 - 1, lo, hi);
      lo = max(lo, 0);
      hi = min(hi, p[6 + d] - 1);
      bad = lo > hi;
      bad |= __shfl_xor(bad, 1);
      if (bad) continue;
      int* o = sb + 4 * p[0];
      if (o[d] >= o[d + 2]) {
        o[d] = lo;
        o[d + 2] = hi + 1;
      } else {
        o[d] = min(o[d], lo);
        o[d + 2] = max(o[d + 2], hi + 1);
      }
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < nbox; k += 64) reinterpret_cast<int4*>(boxes)[(size_t)k * B + b] = sbox[k];
}
}  // namespace

extern "C" int po_grad_boxes(const int32_t* roi, int B, int S, const int32_t* prog, int nprog, int nbox,
                             int32_t* boxes, po_stream_t s) {
  PO_REQUIRE(prog && boxes, "po_grad_boxes: null pointer");
  PO_REQUIRE(B >= 1 && S >= 1 && nprog >= 1 && nbox >= 1, "po_grad_boxes: bad sizes");
  const size_t lds = (size_t)nbox * 16 + (size_t)nprog * 32;
  PO_REQUIRE(lds <= 65536, "po_grad_boxes: %d boxes and %d rows exceed the 64 KB staging limit", nbox, nprog);
  hipLaunchKernelGGL(grad_boxes_k, dim3(B), dim3(64), lds, po::stream_of(s), roi, B, S, prog, nprog, nbox, boxes);
  return po::check_launch("po_grad_boxes");
}

namespace {
// Support boxes of the compact dgrad grids (NetPlan._support / set_support_boxes):
// per entry e and image i < nb, the window of block `win` at org[win][b0 + i]
// dilated by the launch's taps, clipped to the H x W source map, intersected
// with the source block's gradient cone when it has one, written as
// {r0, c0, r1, c1} to the entry's box array dst[e][i].
__global__ __launch_bounds__(64) void support_boxes_k(const int32_t* __restrict__ org, const int32_t* __restrict__ cones,
                                                      const int32_t* __restrict__ prog,
                                                      const unsigned long long* __restrict__ dst, int B) {
  const int e = blockIdx.y;
  const int i = blockIdx.x * 64 + threadIdx.x;
  const int32_t* p = prog + 12 * e;
  const int win = p[0], b0 = p[1], nb = p[2];
  if (i >= nb) return;
  const int dh1 = p[3], dh0 = p[4], dw1 = p[5], dw0 = p[6], H = p[7], W = p[8], w = p[9], cone = p[10];
  const int b = b0 + i;
  const int oy = org[((size_t)win * B + b) * 2], ox = org[((size_t)win * B + b) * 2 + 1];
  int r0 = min(max(oy - dh1, 0), H), c0 = min(max(ox - dw1, 0), W);
  int r1 = min(max(oy + w - dh0, 0), H), c1 = min(max(ox + w - dw0, 0), W);
  if (cone >= 0) {
    const int4 cb = reinterpret_cast<const int4*>(cones)[(size_t)cone * B + b];
    r0 = max(r0, cb.x);
    c0 = max(c0, cb.y);
    r1 = min(r1, cb.z);
    c1 = min(c1, cb.w);
  }
  reinterpret_cast<int4*>(dst[e])[i] = make_int4(r0, c0, r1, c1);
}
}  // namespace

extern "C" int po_support_boxes(const int32_t* org, const int32_t* cones, const int32_t* prog,
                                const unsigned long long* dst, int E, int B, po_stream_t s) {
  PO_REQUIRE(org && prog && dst, "po_support_boxes: null pointer");
  PO_REQUIRE(E >= 1 && B >= 1, "po_support_boxes: bad sizes E=%d B=%d", E, B);
  hipLaunchKernelGGL(support_boxes_k, dim3(po::ceil_div(B, 64), E), dim3(64), 0, po::stream_of(s), org, cones, prog,
                     dst, B);
  return po::check_launch("po_support_boxes");
}
