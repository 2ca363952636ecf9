// First network layer on gfx950: 3 input channels (the NCHW image), 3x3,
// as VALU direct convolution (K = 27 is too short for a matrix-core GEMM), and
// its input gradient, restricted to the patch footprint on the training path.
#include "common.h"
#include "warp_geom.h"

namespace {
// ------------------------------------------------------------------------
// First layer: 3 input channels (NCHW image), 3x3, VALU direct convolution.
// ------------------------------------------------------------------------
// One thread per output pixel.  The weights are read with wave-uniform
// indices straight from global memory, so they arrive through the scalar cache
// as SGPR operands of the FMAs (no LDS broadcast reads); each thread's CO
// outputs go to LDS and the workgroup then writes its 256 pixels x Cout_p
// floats as one contiguous, fully coalesced 16-byte-per-lane stream.
template <int CO>
__global__ __launch_bounds__(256) void first_fwd_k(const float* __restrict__ img, int B, int H, int W,
                                                   int stride, int Ho, int Wo,
                                                   const float* __restrict__ Wt,
                                                   const float* __restrict__ bias, int Cout,
                                                   int Cout_p, int act, float* __restrict__ y,
                                                   uint32_t* __restrict__ amax) {
  constexpr int LS = CO + 1;                         // LDS row stride (bank-conflict-free column writes)
  __shared__ float ys[256 * LS];
  const int64_t npix = (int64_t)B * Ho * Wo;
  const int64_t pbase = (int64_t)blockIdx.x * 256;
  const int64_t p0 = pbase + threadIdx.x;
  const bool live = p0 < npix;
  const int64_t p = live ? p0 : 0;
  const int b = (int)(p / ((int64_t)Ho * Wo));
  const int rem = (int)(p - (int64_t)b * Ho * Wo);
  const int i = rem / Wo, j = rem % Wo;
  float x[27];
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int hi = i * stride - 1 + kh, wi = j * stride - 1 + kw;
        x[c * 9 + kh * 3 + kw] = (hi >= 0 && hi < H && wi >= 0 && wi < W)
                                     ? img[(((size_t)b * 3 + c) * H + hi) * W + wi] : 0.f;
      }
  float vmax = 0.f;
#pragma unroll
  for (int co = 0; co < CO; ++co) {
    float v = 0.f;
    if (co < Cout) {                                 // wave-uniform
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 27; ++k) s += Wt[co * 27 + k] * x[k];
      s += bias ? bias[co] : 0.f;
      v = act ? po::leaky(s) : s;
    }
    vmax = fmaxf(vmax, fabsf(v));
    ys[threadIdx.x * LS + co] = v;
  }
  if (amax) po::amax_commit(amax, live ? vmax : 0.f);
  __syncthreads();
  const int64_t nlive = min((int64_t)256, npix - pbase);
  float* yb = y + pbase * CO;
  for (int f = threadIdx.x; f < nlive * (CO / 4); f += 256) {
    const int px = f / (CO / 4), ch = (f % (CO / 4)) * 4;
    const float* r = ys + px * LS + ch;
    *reinterpret_cast<float4*>(yb + (int64_t)f * 4) = make_float4(r[0], r[1], r[2], r[3]);
  }
}

// Two pixels per thread (p and p + 256 of a 512-pixel block) as the two
// lanes of packed fp32 FMAs (v_pk_fma_f32, the scalar-cache weight broadcast
// to both halves): half the FMA issue slots and half the weight loads per
// pixel of first_fwd_k, same per-pixel summation order (bit-identical).  The
// taps are read through a buffer resource: out-of-image taps read zero from
// the hardware range check instead of branching.  The two 256-pixel halves
// are staged through LDS and stored as two contiguous 16-byte-per-lane streams.
typedef float f2_t __attribute__((ext_vector_type(2)));
// nt: a streaming (non-temporal) store for outputs larger than the caches
__device__ __forceinline__ void po_store4(float* p, float4 v, int nt) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  if (nt)
    __builtin_nontemporal_store((f4v){v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(p));
  else
    *reinterpret_cast<float4*>(p) = v;
}
//
// Composite source (pimg != NULL, po_conv_first_fwd_cmp): the input is the
// patch composite, of which only the quad box of each image's footprint
// (po::quad_box, what po_warp_box_fwd_keyed writes) is in pimg; everywhere
// else it equals img.  A wave whose taps all miss the boxes runs the plain
// loads; a wave with a tap inside a box reads each tap from the tensor that
// holds it (the same values, so the same bits as on the materialised composite).
template <int CO>
__global__ __launch_bounds__(256) void first_fwd2_k(const float* __restrict__ img, int B, int H, int W,
                                                    int stride, int Ho, int Wo,
                                                    const float* __restrict__ Wt,
                                                    const float* __restrict__ bias, int Cout,
                                                    int act, float* __restrict__ y,
                                                    uint32_t* __restrict__ amax,
                                                    const float* __restrict__ pimg,
                                                    const int32_t* __restrict__ roi, int xr, int nt) {
  constexpr int LS = CO + 1;
  __shared__ float ys[256 * LS];
  const int64_t npix = (int64_t)B * Ho * Wo;
  // xr: consecutive pixel blocks on one XCD (the rows above and below a
  // block's are its neighbours' rows: shared in that XCD's L2)
  const int64_t pbase = (int64_t)(xr ? po::xcd_remap() : (int)blockIdx.x) * 512;
  const int tid = threadIdx.x;
  const uint32_t img_bytes = (uint32_t)((int64_t)B * 3 * H * W * 4);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(img), 0, img_bytes, 0x00020000);
  constexpr uint32_t kOOB = 0x80000000u;
  const uint32_t plane = (uint32_t)H * W * 4u;
  f2_t x[27];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int p0 = (int)pbase + q * 256 + tid;      // npix < 2^31 (host check): 32-bit divisions
    const bool live = p0 < (int)npix;
    const int p = live ? p0 : 0;
    const int b = p / (Ho * Wo);
    const int rem = p - b * Ho * Wo;
    const int i = rem / Wo, j = rem - i * Wo;
    const uint32_t ib = (uint32_t)b * 3u * plane;
    po::QBox bx = {0, 0, 0, 0};
    bool touch = false;
    if (pimg) {
      bx = po::quad_box(roi, b, W);
      touch = live && i * stride + 1 >= bx.y0 && i * stride - 1 < bx.y1 && j * stride + 1 >= bx.qx0 &&
              j * stride - 1 < bx.qx1;
    }
    if (!__any(touch)) {
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int hi = i * stride - 1 + kh, wi = j * stride - 1 + kw;
          const bool ok = live && (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
          const uint32_t o = ok ? ib + ((uint32_t)hi * W + wi) * 4u : kOOB;
#pragma unroll
          for (int c = 0; c < 3; ++c)
            x[c * 9 + kh * 3 + kw][q] = __builtin_bit_cast(
                float, __builtin_amdgcn_raw_buffer_load_b32(rs, ok ? o + c * plane : kOOB, 0, 0));
        }
    } else {
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int hi = i * stride - 1 + kh, wi = j * stride - 1 + kw;
          const bool ok = live && (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
          const bool in = hi >= bx.y0 && hi < bx.y1 && wi >= bx.qx0 && wi < bx.qx1;
          const float* src = (in ? pimg : img) + (size_t)b * 3 * H * W + (size_t)hi * W + wi;
#pragma unroll
          for (int c = 0; c < 3; ++c) x[c * 9 + kh * 3 + kw][q] = ok ? src[(size_t)c * H * W] : 0.f;
        }
    }
  }
  f2_t out[CO];
  f2_t vmax = {0.f, 0.f};
#pragma unroll
  for (int co = 0; co < CO; ++co) {
    f2_t v = {0.f, 0.f};
    if (co < Cout) {                                 // wave-uniform
      f2_t s = {0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 27; ++k) s = __builtin_elementwise_fma((f2_t)(Wt[co * 27 + k]), x[k], s);
      s += (f2_t)(bias ? bias[co] : 0.f);
      v = s;
      if (act) {
        v[0] = po::leaky(s[0]);
        v[1] = po::leaky(s[1]);
      }
    }
    vmax[0] = fmaxf(vmax[0], fabsf(v[0]));
    vmax[1] = fmaxf(vmax[1], fabsf(v[1]));
    out[co] = v;
  }
  const bool live1 = pbase + 256 + tid < npix;
  if (amax) po::amax_commit(amax, fmaxf(pbase + tid < npix ? vmax[0] : 0.f, live1 ? vmax[1] : 0.f));
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    if (q) __syncthreads();
#pragma unroll
    for (int co = 0; co < CO; ++co) ys[tid * LS + co] = out[co][q];
    __syncthreads();
    const int64_t hb = pbase + q * 256;
    const int64_t nlive = min((int64_t)256, npix - hb);
    float* yb = y + hb * CO;
    for (int f = tid; f < nlive * (CO / 4); f += 256) {
      const int px = f / (CO / 4), ch = (f % (CO / 4)) * 4;
      const float* r = ys + px * LS + ch;
      po_store4(yb + (int64_t)f * 4, make_float4(r[0], r[1], r[2], r[3]), nt);
    }
  }
}

// The conv + LeakyReLU + 2x2 window rule of one pooled pixel from its 4x4x3
// input patch xa (rows 2py-1.., columns 2px-1..): pooled values to ys_px[co],
// argmax codes packed 4 per word into aw, max |pooled| into vmax.
template <int CO, bool WINO>
__device__ __forceinline__ void pool_conv_px(const float (&xa)[3][4][4], const float* __restrict__ Wt,
                                             const float* __restrict__ bias, int Cout, int act, float* ys_px,
                                             uint32_t (&aw)[CO / 4], float& vmax) {
  // xp[c][r][q] = {x(row 2py-1+r, col 2px-1+q), x(row, col + 1)}: the operand
  // pair of the two outputs (dx = 0, 1) of one output row at tap column q
  f2_t xp[3][4][3];
  // WINO: vw[c][k] = {V[2k], V[2k+1]} of V = B^T d B (row-major 4x4), channel c;
  // the row combinations of B^T run packed over column pairs
  f2_t vw[WINO ? 3 : 1][8];
  if constexpr (WINO) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      f2_t d[4][2], t[4][2];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        d[r][0] = (f2_t){xa[c][r][0], xa[c][r][1]};
        d[r][1] = (f2_t){xa[c][r][2], xa[c][r][3]};
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {                  // t = B^T d
        t[0][h] = d[0][h] - d[2][h];
        t[1][h] = d[1][h] + d[2][h];
        t[2][h] = d[2][h] - d[1][h];
        t[3][h] = d[1][h] - d[3][h];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {                  // V = t B (columns combined)
        // (a0, a1) = t[i][0], (a2, a3) = t[i][1]: {a0 - a2, a1 + a2} and
        // {a2 - a1, a1 - a3}, one v_pk_add_f32 each through its operand-select
        // and negate modifiers (x - y is x + (-y), and IEEE addition commutes:
        // the same values bit for bit)
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,0] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,0]"
            : "=v"(vw[c][2 * i]) : "v"(t[i][0]), "v"(t[i][1]));
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1] neg_lo:[1,0] neg_hi:[0,1]"
            : "=v"(vw[c][2 * i + 1]) : "v"(t[i][0]), "v"(t[i][1]));
      }
    }
  } else {
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 3; ++q) xp[c][r][q] = (f2_t){xa[c][r][q], xa[c][r][q + 1]};
  }
  vmax = 0.f;                 // max|pooled value|: the callers read it from ys_px (fp16x3 slots only)
#pragma unroll
  for (int i = 0; i < CO / 4; ++i) aw[i] = 0u;
#pragma unroll
  for (int co = 0; co < CO; ++co) {
    float bv = 0.f;
    uint32_t code = 0u;
    if (co < Cout) {                                 // wave-uniform
      float v[4];                                    // window positions k = 2 dy + dx
      const float bco = bias ? bias[co] : 0.f;
      if constexpr (WINO) {
        // M = sum over channels of U * V, packed over element pairs; the bias
        // enters through M[1][1] (element 5), which A^T M A adds to all four
        // outputs once
        const f2_t* U2 = reinterpret_cast<const f2_t*>(Wt) + co * 24;
        // {0, bias}: one v_pk_mov_b32 from the scalar bias (two moves otherwise)
        f2_t binit;
        asm("v_pk_mov_b32 %0, 0, %1 op_sel:[0,0]" : "=v"(binit) : "s"((uint64_t)__builtin_bit_cast(uint32_t, bco)));
        f2_t m[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const f2_t init = k == 2 ? binit : (f2_t){0.f, 0.f};
          f2_t acc = __builtin_elementwise_fma(U2[k], vw[0][k], init);
          acc = __builtin_elementwise_fma(U2[8 + k], vw[1][k], acc);
          m[k] = __builtin_elementwise_fma(U2[16 + k], vw[2][k], acc);
        }
        f2_t s0[2], s1[2];                           // A^T M: rows (1 1 1 0), (0 1 -1 -1)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          s0[h] = (m[h] + m[2 + h]) + m[4 + h];
          s1[h] = (m[2 + h] - m[4 + h]) - m[6 + h];
        }
        v[0] = (s0[0][0] + s0[0][1]) + s0[1][0];      // (A^T M) A
        v[1] = (s0[0][1] - s0[1][0]) - s0[1][1];
        v[2] = (s1[0][0] + s1[0][1]) + s1[1][0];
        v[3] = (s1[0][1] - s1[1][0]) - s1[1][1];
      } else {
        f2_t s0 = {0.f, 0.f}, s1 = {0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
          for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
              const f2_t w = (f2_t)(Wt[co * 27 + c * 9 + kh * 3 + kw]);
              s0 = __builtin_elementwise_fma(w, xp[c][kh][kw], s0);
              s1 = __builtin_elementwise_fma(w, xp[c][kh + 1][kw], s1);
            }
        const f2_t bb = (f2_t)bco;
        s0 += bb;
        s1 += bb;
        v[0] = s0[0];
        v[1] = s0[1];
        v[2] = s1[0];
        v[3] = s1[1];
      }
      if (WINO) {
        // the pool before the activation: LeakyReLU is non-decreasing, so the
        // window's max of leaky(v) is leaky(max v), bit for bit, and one
        // activation replaces four.  The window position is the first
        // maximum of v; it differs from the first maximum of leaky(v) only
        // where two negative values round to one leaky value (a tie of the
        // pooled values either way).  Not taken in the direct
        // form, which is bit-identical to conv + po_maxpool2_fwd.
        bv = v[0];
#pragma unroll
        for (int k = 1; k < 4; ++k)
          if (v[k] > bv || isnan(v[k])) { bv = v[k]; code = (uint32_t)k; }
        if (act) bv = po::leaky(bv);
      } else {
        if (act) {
#pragma unroll
          for (int k = 0; k < 4; ++k) v[k] = po::leaky(v[k]);
        }
        bv = v[0];
#pragma unroll
        for (int k = 1; k < 4; ++k)
          if (v[k] > bv || isnan(v[k])) { bv = v[k]; code = (uint32_t)k; }
      }
      if (act) code |= 8u | (bv > 0.f ? 0u : 4u);   // linear conv: no slope to apply
    }
    ys_px[co] = bv;
    aw[co >> 2] |= code << (8 * (co & 3));
  }
}

// First conv (stride 1) with the k=2 stride-2 max pool that follows it fused
// into the epilogue (yolov3-tiny: conv 3->16 @416 then maxpool,
// darknet_v3.py:61-69).  The conv output is never stored: the pool backward
// needs only the window argmax and leaky'(y) at the argmax, which equals
// leaky'(pooled max) (same value).  One thread per pooled pixel: the 4x4x3
// input patch of its 2x2 conv outputs (zero outside the image through the
// buffer range check), the two output rows as packed pairs (v_pk_fma_f32,
// weights from the scalar cache), per output the summation order of
// first_fwd2_k (bit-identical conv values), and po_maxpool2_fwd's window rule
// (first position on ties, NaN wins).  Argmax byte: bits 0-1 window position,
// bit 3 "LeakyReLU mask encoded", bit 2 set when the max is not positive
// (slope 0.1 in the backward).  Pooled floats are staged through LDS for
// fully coalesced 16-byte stores; each thread's CO argmax bytes are one or two
// contiguous 16-byte stores.
// WINO: the conv as Winograd F(2x2,3x3) -- the pooled pixel's 2x2 conv outputs
// are one F(2x2) output tile: V = B^T d B of the 4x4 input patch per channel
// (adds only), 16 products per channel and output channel against Wt = U =
// G g G^T ([CO][3][16], po_conv_first_pool_wino_fwd), Y = A^T M A -- 768
// products per pooled pixel instead of 1728, the same pool rule and argmax
// codes after it.  Not bit-identical to the direct form (another exact
// factorisation of the same sums).
template <int CO, bool WINO>
__global__ __launch_bounds__(256) void first_pool_fwd_k(const float* __restrict__ img, int B, int H, int W,
                                                        int Hp, int Wp, const float* __restrict__ Wt,
                                                        const float* __restrict__ bias, int Cout, int act,
                                                        float* __restrict__ y, int8_t* __restrict__ am,
                                                        uint32_t* __restrict__ amax,
                                                        const float* __restrict__ pimg,
                                                        const int32_t* __restrict__ roi) {
  constexpr int LS = CO + 1;
  __shared__ float ys[256 * LS];
  const int npix = B * Hp * Wp;                     // < 2^31 (host check)
  const int pbase = (int)blockIdx.x * 256;
  const int tid = threadIdx.x;
  const int p0 = pbase + tid;
  const bool live = p0 < npix;
  const int p = live ? p0 : 0;
  const int b = p / (Hp * Wp);
  const int rem = p - b * Hp * Wp;
  const int py = rem / Wp, px = rem - py * Wp;
  const uint32_t img_bytes = (uint32_t)((int64_t)B * 3 * H * W * 4);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(img), 0, img_bytes, 0x00020000);
  constexpr uint32_t kOOB = 0x80000000u;
  const uint32_t plane = (uint32_t)H * W * 4u;
  const uint32_t ib = (uint32_t)b * 3u * plane;
  // composite source: as first_fwd2_k (the 4x4 input window of the pooled pixel)
  po::QBox bx = {0, 0, 0, 0};
  bool touch = false;
  if (pimg) {
    bx = po::quad_box(roi, b, W);
    touch = live && 2 * py + 2 >= bx.y0 && 2 * py - 1 < bx.y1 && 2 * px + 2 >= bx.qx0 && 2 * px - 1 < bx.qx1;
  }
  float xa[3][4][4];
  if (!__any(touch)) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int hi = 2 * py - 1 + r, wi = 2 * px - 1 + q;
        const bool ok = live && (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
        const uint32_t o = ib + ((uint32_t)hi * W + wi) * 4u;
#pragma unroll
        for (int c = 0; c < 3; ++c)
          xa[c][r][q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, ok ? o + c * plane : kOOB, 0, 0));
      }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int hi = 2 * py - 1 + r, wi = 2 * px - 1 + q;
        const bool ok = live && (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
        const bool in = hi >= bx.y0 && hi < bx.y1 && wi >= bx.qx0 && wi < bx.qx1;
        const float* src = (in ? pimg : img) + (size_t)b * 3 * H * W + (size_t)hi * W + wi;
#pragma unroll
        for (int c = 0; c < 3; ++c) xa[c][r][q] = ok ? src[(size_t)c * H * W] : 0.f;
      }
  }
  float vmax;
  uint32_t aw[CO / 4];
  pool_conv_px<CO, WINO>(xa, Wt, bias, Cout, act, ys + tid * LS, aw, vmax);
  if (amax) {                                       // fp16x3 plans only: no VALU spent on it otherwise
#pragma unroll
    for (int co = 0; co < CO; ++co) vmax = fmaxf(vmax, fabsf(ys[tid * LS + co]));
    po::amax_commit(amax, live ? vmax : 0.f);
  }
  if (live) {
    uint4* ap = reinterpret_cast<uint4*>(am + (int64_t)p0 * CO);
#pragma unroll
    for (int i = 0; i < CO / 16; ++i) ap[i] = make_uint4(aw[4 * i], aw[4 * i + 1], aw[4 * i + 2], aw[4 * i + 3]);
  }
  __syncthreads();
  const int nlive = min(256, npix - pbase);
  float* yb = y + (int64_t)pbase * CO;
  for (int f = tid; f < nlive * (CO / 4); f += 256) {
    const int q = f / (CO / 4), ch = (f % (CO / 4)) * 4;
    const float* r = ys + q * LS + ch;
    *reinterpret_cast<float4*>(yb + (int64_t)f * 4) = make_float4(r[0], r[1], r[2], r[3]);
  }
}

// first_pool_fwd_k over 16x16 tiles of pooled pixels: the workgroup stages
// the tile's 34x34x3 input window in LDS with coalesced 16-byte loads (4 per
// thread instead of 48 strided gathers; each input element fetched once per
// tile instead of four times per thread), then each thread reads its 4x4x3
// patch from LDS.  W % 4 == 0 and 16-byte aligned images (host check; else
// first_pool_fwd_k).  Same arithmetic per pixel as first_pool_fwd_k
// (pool_conv_px), so the outputs are bit-identical to it; the LDS window
// aliases the output staging (a barrier between).
template <int CO, bool WINO, bool ACT>
__global__ __launch_bounds__(256) void first_pool_tile_k(const float* __restrict__ img, int B, int H, int W,
                                                         int Hp, int Wp, int tiles_x, int tiles_y,
                                                         const float* __restrict__ Wt,
                                                         const float* __restrict__ bias, int Cout, int act,
                                                         float* __restrict__ y, int8_t* __restrict__ am,
                                                         uint32_t* __restrict__ amax,
                                                         const float* __restrict__ pimg,
                                                         const int32_t* __restrict__ roi, int xr, int nt) {
  constexpr int LS = CO + 1;
  constexpr int TE = 34, TLD = 40;                  // input window rows/columns (2*16 + 2); LDS row: 10 column groups
  static_assert(3 * TE * TLD <= 256 * LS, "input window must fit the output staging");
  __shared__ float ys[256 * LS];
  const int tid = threadIdx.x;
  // xr: consecutive tiles (row-major within an image) on one XCD, so the
  // halo rows and columns neighbouring tiles share hit that XCD's L2
  int t = xr ? po::xcd_remap() : (int)blockIdx.x;
  const int b = t / (tiles_x * tiles_y);
  t -= b * tiles_x * tiles_y;
  const int ty = t / tiles_x, tx = t - ty * tiles_x;
  const int ly = tid >> 4, lx = tid & 15;
  const int py = ty * 16 + ly, px = tx * 16 + lx;
  const bool live = py < Hp && px < Wp;
  const int r0 = 32 * ty - 1, c0 = 32 * tx - 1;     // image row/column of window element (0, 0)
  const uint32_t img_bytes = (uint32_t)((int64_t)B * 3 * H * W * 4);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(img), 0, img_bytes, 0x00020000);
  constexpr uint32_t kOOB = 0x80000000u;
  const uint32_t plane = (uint32_t)H * W * 4u;
  const uint32_t ib = (uint32_t)b * 3u * plane;
  po::QBox bx = {0, 0, 0, 0};
  bool touch = false;                               // workgroup-uniform: the window meets the composite box
  if (pimg) {
    bx = po::quad_box(roi, b, W);
    touch = r0 + TE > bx.y0 && r0 < bx.y1 && c0 + TE > bx.qx0 && c0 < bx.qx1;
  }
  // the window's image columns 32tx-1 .. 32tx+32 lie in the 16-byte column
  // groups 8tx-1 .. 8tx+8 (W % 4 == 0, host check): 10 float4 loads per
  // window row, 102 rows, 4 per thread; a group is entirely inside or outside
  // the image and the quad-widened composite box (both 4-aligned in x)
  float* xs = ys;
  const __amdgpu_buffer_rsrc_t rp =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(pimg ? pimg : img), 0, img_bytes, 0x00020000);
#pragma unroll
  for (int k = 0; k < (3 * TE * 10 + 255) / 256; ++k) {
    const int e = tid + 256 * k;
    const int R = e / 10, g = e - R * 10;           // window row R = c * TE + r, column group g
    const int c = (R >= TE) + (R >= 2 * TE), r = R - c * TE;
    const int hi = r0 + r, wi = 32 * tx - 4 + 4 * g;
    const bool ok = e < 3 * TE * 10 && (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
    const bool in = touch && hi >= bx.y0 && hi < bx.y1 && wi >= bx.qx0 && wi < bx.qx1;
    const uint32_t o = ib + c * plane + ((uint32_t)hi * W + wi) * 4u;
    float4 v;
    if (!touch) {
      v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? o : kOOB, 0, 0));
    } else {
      const float4 vi = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, ok && !in ? o : kOOB, 0, 0));
      const float4 vp = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rp, ok && in ? o : kOOB, 0, 0));
      v = in ? vp : vi;
    }
    // LDS column = image column - (32tx - 4): 16-byte stores
    if (e < 3 * TE * 10) *reinterpret_cast<float4*>(xs + R * TLD + 4 * g) = v;
  }
  __syncthreads();
  float xa[3][4][4];
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) xa[c][r][q] = xs[(c * TE + 2 * ly + r) * TLD + 2 * lx + 3 + q];
  __syncthreads();                                  // ys aliases the window
  float vmax;
  uint32_t aw[CO / 4];
  pool_conv_px<CO, WINO>(xa, Wt, bias, Cout, ACT ? 1 : 0, ys + tid * LS, aw, vmax);   // act == ACT (host)
  if (amax) {                                       // fp16x3 plans only: no VALU spent on it otherwise
#pragma unroll
    for (int co = 0; co < CO; ++co) vmax = fmaxf(vmax, fabsf(ys[tid * LS + co]));
    po::amax_commit(amax, live ? vmax : 0.f);
  }
  const int64_t row0 = ((int64_t)b * Hp + ty * 16) * Wp + tx * 16;   // pixel (ly = 0, lx = 0)
  if (live) {
    uint4* ap = reinterpret_cast<uint4*>(am + (row0 + (int64_t)ly * Wp + lx) * CO);
#pragma unroll
    for (int i = 0; i < CO / 16; ++i) ap[i] = make_uint4(aw[4 * i], aw[4 * i + 1], aw[4 * i + 2], aw[4 * i + 3]);
  }
  __syncthreads();
  const int nx = min(16, Wp - tx * 16), ny = min(16, Hp - ty * 16);
  for (int f = tid; f < 256 * (CO / 4); f += 256) {
    const int q = f / (CO / 4), ch = (f % (CO / 4)) * 4;
    const int qy = q >> 4, qx = q & 15;
    if (qy < ny && qx < nx) {
      const float* r = ys + q * LS + ch;
      po_store4(y + (row0 + (int64_t)qy * Wp + qx) * CO + ch, make_float4(r[0], r[1], r[2], r[3]), nt);
    }
  }
}

template <int CO>
__global__ __launch_bounds__(256) void first_dgrad_k(const float* __restrict__ D, int B, int H, int W,
                                                     int stride, int Ho, int Wo,
                                                     const float* __restrict__ Wt, int Cout,
                                                     int Cout_p, const int32_t* __restrict__ roi,
                                                     float* __restrict__ dimg) {
  __shared__ float ws[CO * 27];
  // roi mode: blockIdx.y = image, blockIdx.x tiles the image's box
  const int b = roi ? (int)blockIdx.y : 0;
  int x0 = 0, y0 = 0, x1 = W, y1 = H;
  if (roi) {
    x0 = roi[4 * b]; y0 = roi[4 * b + 1]; x1 = roi[4 * b + 2]; y1 = roi[4 * b + 3];
    if ((int64_t)blockIdx.x * 256 >= (int64_t)(x1 - x0) * (y1 - y0)) return;   // whole block outside
  }
  for (int t = threadIdx.x; t < CO * 27; t += 256) ws[t] = (t / 27) < Cout ? Wt[t] : 0.f;
  __syncthreads();
  int h, w, bb;
  if (roi) {
    const int q = blockIdx.x * 256 + threadIdx.x;
    const int bw = x1 - x0;
    if (q >= bw * (y1 - y0)) return;
    h = y0 + q / bw;
    w = x0 + q % bw;
    bb = b;
  } else {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= (int64_t)B * H * W) return;
    bb = (int)(p / ((int64_t)H * W));
    const int rem = (int)(p - (int64_t)bb * H * W);
    h = rem / W;
    w = rem % W;
  }
  const int b_ = bb;
  float d0 = 0.f, d1 = 0.f, d2 = 0.f;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int th = h + 1 - kh;
    if (th < 0 || th % stride) continue;
    const int ho = th / stride;
    if (ho >= Ho) continue;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int tw = w + 1 - kw;
      if (tw < 0 || tw % stride) continue;
      const int wo = tw / stride;
      if (wo >= Wo) continue;
      const float* dp = D + (((size_t)b_ * Ho + ho) * Wo + wo) * Cout_p;
#pragma unroll
      for (int co4 = 0; co4 < CO; co4 += 4) {
        const float4 g = *reinterpret_cast<const float4*>(dp + co4);
        const float gg[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float* wc = ws + (co4 + u) * 27 + kh * 3 + kw;
          d0 += gg[u] * wc[0];
          d1 += gg[u] * wc[9];
          d2 += gg[u] * wc[18];
        }
      }
    }
  }
  const size_t plane = (size_t)H * W;
  float* o = dimg + (size_t)b_ * 3 * plane + (size_t)h * W + w;
  o[0] = d0;
  o[plane] = d1;
  o[2 * plane] = d2;
}
}  // namespace

namespace {
int first_fwd(const float* img, const float* pimg, const int32_t* roi, int B, int H, int W, int stride, const float* Wt,
              const float* bias, int Cout, int Cout_p, int act, float* y, uint32_t* amax, po_stream_t s) {
  PO_REQUIRE(img && Wt && y, "po_conv_first_fwd: null pointer");
  PO_REQUIRE(stride == 1 || stride == 2, "po_conv_first_fwd: stride %d", stride);
  PO_REQUIRE(Cout > 0 && Cout <= 64 && Cout_p % 4 == 0 && Cout_p >= Cout, "po_conv_first_fwd: Cout=%d Cout_p=%d", Cout, Cout_p);
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const int64_t n = (int64_t)B * Ho * Wo;
  dim3 grid(po::ceil_div(n, 256));
  hipStream_t st = po::stream_of(s);
  const int CO = Cout_p <= 16 ? 16 : (Cout_p <= 32 ? 32 : 64);
  PO_REQUIRE(Cout_p == CO, "po_conv_first_fwd: Cout_p must be 16, 32 or 64 (got %d)", Cout_p);
  PO_REQUIRE((int64_t)B * 3 * H * W * 4 < (1LL << 31) && n + 512 < (1LL << 31),
             "po_conv_first_fwd: image batch must be < 2 GiB");
  PO_REQUIRE(!pimg || (roi && CO <= 32 && H == W), "po_conv_first_fwd_cmp: needs roi, a square image and Cout_p <= 32");
  dim3 grid2(po::ceil_div(n, 512));
  // the XCD remap cuts this launch's fetched bytes 229 -> 68 MB (yolov3 B=16)
  // but measured 201 -> 206 us: off unless ADVPATCH_FIRST_XCD=1
  // (profiles/r05/first_xcd_ab.txt)
  static const int xr = [] {
    const char* e = getenv("ADVPATCH_FIRST_XCD");
    return (e && e[0] == '1') ? 1 : 0;
  }();
  static const int nt = [] {
    const char* e = getenv("ADVPATCH_FIRST_NT");
    return (e && e[0] == '1') ? 1 : 0;
  }();
  if (CO == 16)
    hipLaunchKernelGGL(first_fwd2_k<16>, grid2, dim3(256), 0, st, img, B, H, W, stride, Ho, Wo, Wt, bias, Cout, act, y, amax,
                       pimg, roi, xr, nt);
  else if (CO == 32)
    hipLaunchKernelGGL(first_fwd2_k<32>, grid2, dim3(256), 0, st, img, B, H, W, stride, Ho, Wo, Wt, bias, Cout, act, y, amax,
                       pimg, roi, xr, nt);
  else
    hipLaunchKernelGGL(first_fwd_k<64>, grid, dim3(256), 0, st, img, B, H, W, stride, Ho, Wo, Wt, bias, Cout, Cout_p, act, y, amax);
  return po::check_launch("po_conv_first_fwd");
}

int first_pool_fwd(const float* img, const float* pimg, const int32_t* roi, int B, int H, int W, const float* Wt,
                   const float* bias, int Cout, int Cout_p, int act, float* y, int8_t* argmax, uint32_t* amax,
                   po_stream_t s, bool wino = false) {
  PO_REQUIRE(img && Wt && y && argmax, "po_conv_first_pool_fwd: null pointer");
  static const bool lt = [] {
    const char* e = getenv("ADVPATCH_FIRST_TILE");
    return !(e && e[0] == '0');
  }();
  static const int xr = [] {
    const char* e = getenv("ADVPATCH_FIRST_XCD");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  static const int nt = [] {
    const char* e = getenv("ADVPATCH_FIRST_NT");
    return (e && e[0] == '1') ? 1 : 0;
  }();
  PO_REQUIRE((Cout_p == 16 || Cout_p == 32) && Cout > 0 && Cout <= Cout_p,
             "po_conv_first_pool_fwd: Cout_p must be 16 or 32 (got %d, Cout %d)", Cout_p, Cout);
  PO_REQUIRE(B > 0 && H >= 2 && W >= 2, "po_conv_first_pool_fwd: bad size B=%d H=%d W=%d", B, H, W);
  PO_REQUIRE(!pimg || (roi && H == W), "po_conv_first_pool_fwd_cmp: needs roi and a square image");
  const int Hp = H / 2, Wp = W / 2;
  const int64_t n = (int64_t)B * Hp * Wp;
  PO_REQUIRE((int64_t)B * 3 * H * W * 4 < (1LL << 31) && n + 256 < (1LL << 31),
             "po_conv_first_pool_fwd: image batch must be < 2 GiB");
  hipStream_t st = po::stream_of(s);
  if (lt && W % 4 == 0 && ((uintptr_t)img & 15) == 0 && ((uintptr_t)pimg & 15) == 0) {   // 16x16 pooled tiles
    const int tx = (Wp + 15) / 16, ty = (Hp + 15) / 16;
    PO_REQUIRE((int64_t)B * tx * ty < (1LL << 31), "po_conv_first_pool_fwd: too many tiles");
    dim3 gt((unsigned)(B * tx * ty));
#define PO_FPT(CO_, WI_, AC_)                                                                                   \
  hipLaunchKernelGGL((first_pool_tile_k<CO_, WI_, AC_>), gt, dim3(256), 0, st, img, B, H, W, Hp, Wp, tx, ty, Wt,     \
                     bias, Cout, act, y, argmax, amax, pimg, roi, xr, nt)
    // the activation as a template argument: no per-channel selects between the two forms
    if (Cout_p == 16) {
      if (wino) { if (act) PO_FPT(16, true, true); else PO_FPT(16, true, false); }
      else { if (act) PO_FPT(16, false, true); else PO_FPT(16, false, false); }
    } else {
      if (wino) { if (act) PO_FPT(32, true, true); else PO_FPT(32, true, false); }
      else { if (act) PO_FPT(32, false, true); else PO_FPT(32, false, false); }
    }
#undef PO_FPT
    return po::check_launch("po_conv_first_pool_fwd");
  }
  dim3 grid(po::ceil_div(n, 256));
  if (wino) {
    if (Cout_p == 16)
      hipLaunchKernelGGL((first_pool_fwd_k<16, true>), grid, dim3(256), 0, st, img, B, H, W, Hp, Wp, Wt, bias, Cout, act,
                         y, argmax, amax, pimg, roi);
    else
      hipLaunchKernelGGL((first_pool_fwd_k<32, true>), grid, dim3(256), 0, st, img, B, H, W, Hp, Wp, Wt, bias, Cout, act,
                         y, argmax, amax, pimg, roi);
  } else if (Cout_p == 16) {
    hipLaunchKernelGGL((first_pool_fwd_k<16, false>), grid, dim3(256), 0, st, img, B, H, W, Hp, Wp, Wt, bias, Cout, act,
                       y, argmax, amax, pimg, roi);
  } else {
    hipLaunchKernelGGL((first_pool_fwd_k<32, false>), grid, dim3(256), 0, st, img, B, H, W, Hp, Wp, Wt, bias, Cout, act,
                       y, argmax, amax, pimg, roi);
  }
  return po::check_launch("po_conv_first_pool_fwd");
}
}  // namespace

extern "C" int po_conv_first_fwd(const float* img, int B, int H, int W, int stride, const float* Wt,
                                 const float* bias, int Cout, int Cout_p, int act, float* y,
                                 uint32_t* amax, po_stream_t s) {
  return first_fwd(img, nullptr, nullptr, B, H, W, stride, Wt, bias, Cout, Cout_p, act, y, amax, s);
}

extern "C" int po_conv_first_fwd_cmp(const float* img, const float* pimg, const int32_t* roi, int B, int H, int W,
                                     int stride, const float* Wt, const float* bias, int Cout, int Cout_p, int act,
                                     float* y, uint32_t* amax, po_stream_t s) {
  PO_REQUIRE(pimg, "po_conv_first_fwd_cmp: null composite");
  return first_fwd(img, pimg, roi, B, H, W, stride, Wt, bias, Cout, Cout_p, act, y, amax, s);
}

extern "C" int po_conv_first_pool_fwd(const float* img, int B, int H, int W, const float* Wt, const float* bias,
                                      int Cout, int Cout_p, int act, float* y, int8_t* argmax, uint32_t* amax,
                                      po_stream_t s) {
  return first_pool_fwd(img, nullptr, nullptr, B, H, W, Wt, bias, Cout, Cout_p, act, y, argmax, amax, s);
}

extern "C" int po_conv_first_pool_fwd_cmp(const float* img, const float* pimg, const int32_t* roi, int B, int H, int W,
                                          const float* Wt, const float* bias, int Cout, int Cout_p, int act, float* y,
                                          int8_t* argmax, uint32_t* amax, po_stream_t s) {
  PO_REQUIRE(pimg, "po_conv_first_pool_fwd_cmp: null composite");
  return first_pool_fwd(img, pimg, roi, B, H, W, Wt, bias, Cout, Cout_p, act, y, argmax, amax, s);
}

extern "C" int po_conv_first_pool_wino_fwd(const float* img, int B, int H, int W, const float* U, const float* bias,
                                           int Cout, int Cout_p, int act, float* y, int8_t* argmax, uint32_t* amax,
                                           po_stream_t s) {
  return first_pool_fwd(img, nullptr, nullptr, B, H, W, U, bias, Cout, Cout_p, act, y, argmax, amax, s, true);
}

extern "C" int po_conv_first_pool_wino_fwd_cmp(const float* img, const float* pimg, const int32_t* roi, int B, int H,
                                               int W, const float* U, const float* bias, int Cout, int Cout_p,
                                               int act, float* y, int8_t* argmax, uint32_t* amax, po_stream_t s) {
  PO_REQUIRE(pimg, "po_conv_first_pool_wino_fwd_cmp: null composite");
  return first_pool_fwd(img, pimg, roi, B, H, W, U, bias, Cout, Cout_p, act, y, argmax, amax, s, true);
}

extern "C" int po_conv_first_dgrad(const float* D, int B, int H, int W, int stride, const float* Wt,
                                   int Cout, int Cout_p, const int32_t* roi, float* d_img,
                                   po_stream_t s) {
  PO_REQUIRE(D && Wt && d_img, "po_conv_first_dgrad: null pointer");
  PO_REQUIRE(stride == 1 || stride == 2, "po_conv_first_dgrad: stride %d", stride);
  const int CO = Cout_p <= 16 ? 16 : (Cout_p <= 32 ? 32 : 64);
  PO_REQUIRE(Cout_p == CO && Cout <= Cout_p, "po_conv_first_dgrad: Cout_p must be 16, 32 or 64 (got %d)", Cout_p);
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  // with a roi, blockIdx.y = image and blockIdx.x covers up to the whole image
  // (blocks past the image's box exit at once)
  const int64_t n = roi ? (int64_t)H * W : (int64_t)B * H * W;
  dim3 grid(po::ceil_div(n, 256), roi ? B : 1);
  hipStream_t st = po::stream_of(s);
  if (CO == 16)
    hipLaunchKernelGGL(first_dgrad_k<16>, grid, dim3(256), 0, st, D, B, H, W, stride, Ho, Wo, Wt, Cout, Cout_p, roi, d_img);
  else if (CO == 32)
    hipLaunchKernelGGL(first_dgrad_k<32>, grid, dim3(256), 0, st, D, B, H, W, stride, Ho, Wo, Wt, Cout, Cout_p, roi, d_img);
  else
    hipLaunchKernelGGL(first_dgrad_k<64>, grid, dim3(256), 0, st, D, B, H, W, stride, Ho, Wo, Wt, Cout, Cout_p, roi, d_img);
  return po::check_launch("po_conv_first_dgrad");
}
