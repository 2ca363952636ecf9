// Pieces shared by the two implicit-GEMM convolution kernels of po_conv:
//   conv_k    (conv_igemm.hip) exact fp32 operands on v_mfma_f32_32x32x2_f32;
//   conv_h3_k (conv_h3.hip)    fp32 operands split into two fp16 pieces under a
//                              per-tensor power-of-two scale, three
//                              v_mfma_f32_32x32x16_f16 products, fp32 accumulate.
// Both accumulate 32x32 tiles with the same C/D register layout
// (row = (e&3) + 8*(e>>2) + 4*(lane>>5), col = lane&31), so the epilogue, the
// split-K partial store and the split-K reduction are common.
#pragma once
#include "common.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace po {

struct ConvArgs {
  const float* in;
  const void* W;                // fp32 [N][ntaps][Cin_p]  or  fp16 [2][N][ntaps][Cin_p] (prec 1)
  const void* Wf;               // optional (prec 1): the same fp16 weights in MFMA fragment order
  const float* bias;
  float* y;
  const float* res;
  float* sum;
  const float* mask;
  float* y2;
  const float* mask2;
  const int32_t* in_org;        // window origins [B,2] (NULL: full map)
  const int32_t* out_org;
  const int32_t* gbox;          // optional per-image boxes [B][4] (r0, c0, r1, c1) of the destination:
                                // only grid points whose output pixel lies in the box are computed
  float* ws;                    // split-K partials [ksplit][M][N] (ksplit > 1)
  int32_t* tile_ctr;            // split-K arrival counters per output tile (conv_k's in-launch reduction; NULL: none)
  int tile_ctr_n;
  const uint32_t* in_amax;      // prec 1: max|in| slot (float bits)
  uint32_t* y_amax;             // optional max|output| slots
  uint32_t* sum_amax;
  uint32_t* y2_amax;
  uint32_t* ybits;              // optional: sign bits (y > 0) of y_out, [pixel][Cout_p/32] words
  const uint32_t* mbits;        // optional: leaky mask as sign bits (replaces mask)
  const uint32_t* m2bits;       //                                   (replaces mask2)
  int prec, w_shift;            // prec 1: weights pre-scaled by 2^w_shift
  int ksplit;
  int B, Hin, Win, Cin_p, Hout, Wout, Cout_p, Hg, Wg;
  int in_step, out_step, out_oy, out_ox;
  int ntaps, N, act, accumulate;
  int M, ntiles_n;
  int mrows;                    // GEMM rows per image: Hg*Wg, or fewer with gbox (a compact grid over each
                                // image's box of at most mrows points: see grid_point)
  float* pool_y;                // optional: k=2 stride-2 max pool of the output fused into the epilogue
  int8_t* pool_am;              //   (pool output, argmax bytes); the grid runs in pool order
  uint32_t in_bytes, w_bytes;   // buffer-resource extents (< 2^31)
  // taps form a rectangular grid: tap t = th*tkw + tw -> (dh0 + th*sdh, dw0 + tw*sdw)
  int tkw, dh0, dw0, sdh, sdw;
  // exact division by mrows and Wg for 0 <= n < 2^31 (host: po::div_magic):
  // n / d = (n * mg) >> sh, no runtime integer-division sequence on the device
  uint32_t mg_rows, mg_wg;
  int sh_rows, sh_wg;
  // the same for the Winograd 2x2-tile grid of tile 70 (Ht*Wt tiles per image, Wt per row)
  uint32_t mg_tiles, mg_wt;
  int sh_tiles, sh_wt;
  // and its unit decomposition (units per split-K slice, n-blocks, slices)
  uint32_t mg_mn, mg_ntn, mg_ks;
  int sh_mn, sh_ntn, sh_ks;
};

// d >= 1: mg = ceil(2^(31+l) / d) < 2^32, sh = 31 + l, l = ceil(log2 d)
inline void div_magic(int d, uint32_t& mg, int& sh) {
  int l = 0;
  while ((1LL << l) < d) ++l;
  mg = (uint32_t)(((1ULL << (31 + l)) + (uint64_t)d - 1) / (uint64_t)d);
  sh = 31 + l;
}
__device__ __forceinline__ int div_by(int n, uint32_t mg, int sh) {
  return (int)(((uint64_t)(uint32_t)n * mg) >> sh);
}

// Input scale exponent of a prec-1 launch: the input is multiplied by 2^e
// (exact) so that its largest magnitude lies in [2^13, 2^14) — inside fp16's
// range with 2 binades of headroom, while the low piece of every element that
// matters stays far above fp16's subnormal floor.
__device__ __forceinline__ int input_shift(const ConvArgs& a) {
  if (a.prec != 1) return 0;
  const uint32_t bits = amax_read(a.in_amax);
  const int e = (int)((bits >> 23) & 0xff) - 127;      // amax in [2^e, 2^(e+1)) (normal)
  return min(max(13 - e, -120), 120);
}

// ---- launch-grid enumeration.  GEMM row m is image b = m / mrows and, in
// that image, grid point l = m % mrows: row-major over the whole Hg x Wg grid
// (mrows = Hg*Wg), or (a.gbox set) row-major over the image's box only, the
// rows past the box's area computing nothing (mrows < Hg*Wg when every box is
// known to hold at most mrows points: the launch has no dead rows to spare).  Grid point (i, j) writes destination pixel
// (i*out_step + out_oy, j*out_step + out_ox).
struct GridBox {
  int i0, j0, h, w;
};
// first i with i*step + off >= lo;  one past the last i < n with i*step + off < hi
__device__ __forceinline__ int grid_lo(int lo, int off, int step) {
  const int d = lo - off;
  return d <= 0 ? 0 : (d + step - 1) / step;
}
__device__ __forceinline__ int grid_hi(int hi, int off, int step, int n) {
  const int d = hi - 1 - off;
  return d < 0 ? 0 : min(n, d / step + 1);
}
__device__ __forceinline__ GridBox grid_box(const ConvArgs& a, int b) {
  const int4 bx = reinterpret_cast<const int4*>(a.gbox)[b];
  const int i0 = grid_lo(bx.x, a.out_oy, a.out_step), i1 = grid_hi(bx.z, a.out_oy, a.out_step, a.Hg);
  const int j0 = grid_lo(bx.y, a.out_ox, a.out_step), j1 = grid_hi(bx.w, a.out_ox, a.out_step, a.Wg);
  return {i0, j0, max(i1 - i0, 0), max(j1 - j0, 0)};
}
// GEMM row m -> image b and grid point (i, j); false: the row computes nothing
__device__ __forceinline__ bool grid_point(const ConvArgs& a, int m, int& b, int& i, int& j) {
  const int HgWg = a.mrows;
  if (m >= a.M) {
    b = i = j = 0;
    return false;
  }
  b = div_by(m, a.mg_rows, a.sh_rows);
  const int l = m - b * HgWg;
  if (a.pool_y) {          // pool order: rows 4w .. 4w+3 are the 2x2 window w (row-major windows)
    const int w = l >> 2, k = l & 3, wp = a.Wg >> 1;
    const int i2 = w / wp;
    i = 2 * i2 + (k >> 1);
    j = 2 * (w - i2 * wp) + (k & 1);
    return true;
  }
  if (!a.gbox) {
    i = div_by(l, a.mg_wg, a.sh_wg);
    j = l - i * a.Wg;
    return true;
  }
  const GridBox g = grid_box(a, b);
  if (l >= g.h * g.w) {
    i = j = 0;
    return false;
  }
  const int q = l / g.w;
  i = g.i0 + q;
  j = g.j0 + (l - q * g.w);
  return true;
}
// does the tile of GEMM rows [m0, m0 + rows) hold a row that computes something?
__device__ __forceinline__ bool tile_live(const ConvArgs& a, int m0, int rows) {
  if (!a.gbox) return true;
  const int HgWg = a.mrows;
  const int m1 = min(m0 + rows, a.M);
  for (int b = m0 / HgWg; b * HgWg < m1; ++b) {
    const GridBox g = grid_box(a, b);
    if (max(m0 - b * HgWg, 0) < g.h * g.w) return true;
  }
  return false;
}

// Raw partial sums of one split-K slice (the reduction applies the epilogue)
template <int TM, int TN>
__device__ __forceinline__ void store_partials(const ConvArgs& a, const floatx16 (&acc)[TM][TN], int m0, int n0,
                                               int wm, int wn, int lane) {
  float* ws = a.ws + (size_t)blockIdx.y * a.M * a.N;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * TN * 32 + j * 32 + (lane & 31);
      if (n >= a.N) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wm * TM * 32 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        if (m < a.M) ws[(size_t)m * a.N + n] = acc[i][j][e];
      }
    }
}

// leaky'(.) factors of 4 consecutive channels n..n+3 from a sign-bit word
__device__ __forceinline__ float4 leaky_grad_bits(uint32_t w, int n) {
  const uint32_t b = w >> (n & 31);
  return make_float4((b & 1) ? 1.f : 0.1f, (b & 2) ? 1.f : 0.1f, (b & 4) ? 1.f : 0.1f, (b & 8) ? 1.f : 0.1f);
}

// Epilogue of a conv with its k=2 stride-2 max pool fused (ConvArgs.pool_y;
// pool-order grid: GEMM rows 4w..4w+3 are the 2x2 window w).  Each wave stages
// one 32x32 accumulator tile through its LDS slot as conv_epilogue does; the
// lane whose rows are window position 0 (row & 3 == 0) reads the window's four
// rows, applies bias + activation to each exactly as conv_epilogue would, then
// po_maxpool2_fwd's rule (first position on ties, NaN wins), and writes the
// pooled value and the argmax byte (bit 3 set and bit 2 = max <= 0 for a leaky
// conv: the LeakyReLU slope of the unstored output, see
// po_conv_first_pool_fwd).  The conv output itself is not stored.
template <int BM, int TM, int TN>
__device__ __forceinline__ void conv_pool_epilogue(const ConvArgs& a, const floatx16 (&acc)[TM][TN], float* smem,
                                                   int* dst_pix, int m0, int n0, int wm, int wn, int sh,
                                                   bool active) {
  const int tid = threadIdx.x, lane = tid & 63, wave = (tid >> 6) & 3;
  if (tid < BM) {
    int b, i, j;
    dst_pix[tid] = grid_point(a, m0 + tid, b, i, j) ? (b * a.Hout + i) * a.Wout + j : -1;
  }
  __syncthreads();
  float* scr = smem + wave * 1024;
  const int rr = lane >> 3, cc = (lane & 7) * 4;
  float my = 0.f;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (!active) break;
#pragma unroll
      for (int e = 0; e < 16; ++e)
        scr[((e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)) * 32 + (lane & 31)] = acc[i][j][e];
      __builtin_amdgcn_wave_barrier();
      const int n = n0 + wn * TN * 32 + j * 32 + cc;
      float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (a.bias && n < a.N) bv = *reinterpret_cast<const float4*>(a.bias + n);
      if ((rr & 3) == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = rr + 8 * q;
          const int pix = dst_pix[wm * TM * 32 + i * 32 + row];
          if (pix < 0 || n >= a.N) continue;
          float pv[4] = {0.f, 0.f, 0.f, 0.f};
          uint32_t arg[4] = {0u, 0u, 0u, 0u};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float4 vk = *reinterpret_cast<const float4*>(scr + (row + k) * 32 + cc);
            float x[4] = {__builtin_ldexpf(vk.x, -sh) + bv.x, __builtin_ldexpf(vk.y, -sh) + bv.y,
                          __builtin_ldexpf(vk.z, -sh) + bv.z, __builtin_ldexpf(vk.w, -sh) + bv.w};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              x[c] = leaky_or_id(x[c], act_slope(a.act));
              if (k == 0 || x[c] > pv[c] || isnan(x[c])) { pv[c] = x[c]; arg[c] = (uint32_t)k; }
            }
          }
          uint32_t code = 0u;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            if (a.act) arg[c] |= 8u | (pv[c] > 0.f ? 0u : 4u);
            if (n + c >= a.N) { pv[c] = 0.f; arg[c] = 0u; }
            code |= arg[c] << (8 * c);
            my = fmaxf(my, fabsf(pv[c]));
          }
          // pixel (b, i, j) of window position 0 (i, j even) -> pooled pixel (b, i/2, j/2)
          const int Wo = a.Wout, Ho = a.Hout;
          const int bimg = pix / (Ho * Wo), rem = pix - bimg * Ho * Wo;
          const int pi = rem / Wo, pj = rem - pi * Wo;
          const uint32_t po = (((uint32_t)bimg * (Ho >> 1) + (pi >> 1)) * (Wo >> 1) + (pj >> 1)) * a.Cout_p + n;
          *reinterpret_cast<float4*>(a.pool_y + po) = make_float4(pv[0], pv[1], pv[2], pv[3]);
          *reinterpret_cast<uint32_t*>(a.pool_am + po) = code;
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  if (a.y_amax) amax_commit(a.y_amax, my);
}

// Epilogue.  Each wave stages one 32x32 accumulator tile at a time through a
// private 4 KB slot of `smem` (the k-loop buffers are free by now), then every
// lane handles 4 consecutive channels of a row: 16-byte loads of
// bias/mask/res and 16-byte stores of y/sum/y2, 128 contiguous bytes per row.
// v = acc * 2^-sh + bias (sh = 0 for fp32 operands; ldexp is exact).
// Waves 0..3 hold the accumulators; in a warp-specialized launch the other
// waves (active = false) only take part in the barrier and the slot commits.
template <int BM, int TM, int TN>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, const floatx16 (&acc)[TM][TN], float* smem,
                                              int* dst_pix, int m0, int n0, int wm, int wn, int sh,
                                              bool active = true, bool fill_dst = true) {
  if constexpr (TM * TN <= 4) {     // pooled launches: tiles up to 128x128 (host check)
    if (a.pool_y) {
      conv_pool_epilogue<BM, TM, TN>(a, acc, smem, dst_pix, m0, n0, wm, wn, sh, active);
      return;
    }
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = (tid >> 6) & 3;
  if (fill_dst && tid < BM) {     // else the caller has written dst_pix (2-D tiles)
    int b, i, j;
    dst_pix[tid] = grid_point(a, m0 + tid, b, i, j)
                       ? (b * a.Hout + i * a.out_step + a.out_oy) * a.Wout + j * a.out_step + a.out_ox
                       : -1;
  }
  __syncthreads();
  float* scr = smem + wave * 1024;
  const int rr = lane >> 3, cc = (lane & 7) * 4;
  float my = 0.f, ms = 0.f, my2 = 0.f;
  // the bias of every column tile, requested before the first store (a load
  // issued after a store waits for it on the shared vmcnt)
  float4 bvs[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * TN * 32 + j * 32 + cc;
    bvs[j] = (a.bias && n < a.N) ? *reinterpret_cast<const float4*>(a.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (!active) break;
#pragma unroll
      for (int e = 0; e < 16; ++e)
        scr[((e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)) * 32 + (lane & 31)] = acc[i][j][e];
      __builtin_amdgcn_wave_barrier();
      const int n = n0 + wn * TN * 32 + j * 32 + cc;
      const float4 bv = bvs[j];
      const int wpp = a.Cout_p >> 5;            // sign-bit words per pixel (bits need Cout_p % 32 == 0)
      // load phase: the rows' shortcut operand, accumulated destination and
      // mask words, all before the first store (gfx9 counts stores and loads
      // on one counter: a load issued after a store waits for that store)
      int pixq[4];
      float4 pres[4], pold[4];
      uint32_t pmw[4], pm2w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        pixq[q] = dst_pix[wm * TM * 32 + i * 32 + rr + 8 * q];
        pres[q] = pold[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        pmw[q] = pm2w[q] = 0u;
        if (pixq[q] >= 0 && n < a.N) {
          const uint32_t o = (uint32_t)pixq[q] * (uint32_t)a.Cout_p + n;      // < 2^31 (po_conv host check)
          const uint32_t wo = (uint32_t)pixq[q] * wpp + (n >> 5);
          if (a.res) pres[q] = *reinterpret_cast<const float4*>(a.res + o);
          if (a.accumulate) pold[q] = *reinterpret_cast<const float4*>(a.y + o);
          if (a.mbits) pmw[q] = a.mbits[wo];
          if (a.y2 && a.m2bits) pm2w[q] = a.m2bits[wo];
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = rr + 8 * q;
        const float4 v = *reinterpret_cast<const float4*>(scr + row * 32 + cc);
        const int pix = pixq[q];
        const bool live = pix >= 0 && n < a.N;
        uint32_t nib = 0;
        if (live) {
          const uint32_t o = (uint32_t)pix * (uint32_t)a.Cout_p + n;
          float x[4] = {__builtin_ldexpf(v.x, -sh) + bv.x, __builtin_ldexpf(v.y, -sh) + bv.y,
                        __builtin_ldexpf(v.z, -sh) + bv.z, __builtin_ldexpf(v.w, -sh) + bv.w};
#pragma unroll
          for (int c = 0; c < 4; ++c) x[c] = leaky_or_id(x[c], act_slope(a.act));
          if (a.accumulate) {
            const float4 p = pold[q];
            x[0] += p.x; x[1] += p.y; x[2] += p.z; x[3] += p.w;
          }
          float4 out = make_float4(x[0], x[1], x[2], x[3]);
          if (a.mbits) {
            const float4 g = leaky_grad_bits(pmw[q], n);
            out = make_float4(x[0] * g.x, x[1] * g.y, x[2] * g.z, x[3] * g.w);
          } else if (a.mask) {
            const float4 mk = *reinterpret_cast<const float4*>(a.mask + o);
            out = make_float4(x[0] * leaky_grad(mk.x), x[1] * leaky_grad(mk.y), x[2] * leaky_grad(mk.z),
                              x[3] * leaky_grad(mk.w));
          }
          if (a.y) *reinterpret_cast<float4*>(a.y + o) = out;     // NULL: only signs/sum wanted
          nib = (out.x > 0.f ? 1u : 0u) | (out.y > 0.f ? 2u : 0u) | (out.z > 0.f ? 4u : 0u) | (out.w > 0.f ? 8u : 0u);
          if (a.y_amax)        // max|x| slots: fp16x3 plans only (no VALU spent on them otherwise)
            my = fmaxf(my, fmaxf(fmaxf(fabsf(out.x), fabsf(out.y)), fmaxf(fabsf(out.z), fabsf(out.w))));
          if (a.res) {
            const float4 r = pres[q];
            const float4 sm = make_float4(x[0] + r.x, x[1] + r.y, x[2] + r.z, x[3] + r.w);
            *reinterpret_cast<float4*>(a.sum + o) = sm;
            if (a.sum_amax) ms = fmaxf(ms, fmaxf(fmaxf(fabsf(sm.x), fabsf(sm.y)), fmaxf(fabsf(sm.z), fabsf(sm.w))));
          }
          if (a.y2) {
            float4 g;
            if (a.m2bits) {
              g = leaky_grad_bits(pm2w[q], n);
            } else {
              const float4 mk = *reinterpret_cast<const float4*>(a.mask2 + o);
              g = make_float4(leaky_grad(mk.x), leaky_grad(mk.y), leaky_grad(mk.z), leaky_grad(mk.w));
            }
            const float4 o2 = make_float4(x[0] * g.x, x[1] * g.y, x[2] * g.z, x[3] * g.w);
            *reinterpret_cast<float4*>(a.y2 + o) = o2;
            if (a.y2_amax) my2 = fmaxf(my2, fmaxf(fmaxf(fabsf(o2.x), fabsf(o2.y)), fmaxf(fabsf(o2.z), fabsf(o2.w))));
          }
        }
        if (a.ybits) {
          // the 8 lanes of a row hold channels n0' .. n0' + 31 of one word: OR their nibbles
          uint32_t w = nib << (4 * (lane & 7));
          w = or_group_down<8>(w);
          if (live && (lane & 7) == 0) a.ybits[(uint32_t)pix * wpp + (n >> 5)] = w;
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  if (a.y_amax) amax_commit(a.y_amax, my);
  if (a.sum_amax) amax_commit(a.sum_amax, ms);
  if (a.y2_amax) amax_commit(a.y2_amax, my2);
}

// conv_h3.hip: launch of the split-precision kernel for tile (bm, bn, bk)
// (the split-K reduction, when a.ksplit > 1, is launched by the caller)
// (staging 1: the LDS-DMA multi-stage kernel; 2: the halo kernel for
// stride-1 3x3 convs on full maps; 3: the 2-D tile halo kernel for stride-1/2
// 3x3 convs on full maps; 4: the same with fragment-ordered weights read from
// global memory)
int launch_h3(const ConvArgs& a, hipStream_t st, int bm, int bn, int bk, int staging);

// conv_wino.hip: the exact-fp32 Winograd F(2x2,3x3) kernel (tile 61); U =
// the launch's transformed weights (po_conv_desc.Wwino)
int launch_wino(const ConvArgs& a, const float* U, hipStream_t st, int bm, int waves, bool sched = false,
                bool vec = false, bool small_lds = false);
// tiles 67/68: 64 tiles x 64 channels per 512-thread workgroup, pipelined k-loop
// (68: the two waves of a SIMD staggered)
int launch_wino4(const ConvArgs& a, const float* U, hipStream_t st, bool stagger);
int launch_wino5(const ConvArgs& a, const float* U, hipStream_t st);
// tile 71 (conv_wino6.hip): Winograd F(4x4,3x3), persistent; U6 = po_conv_desc.Wwino6
int launch_wino6(const ConvArgs& a, const float* U6, hipStream_t st, float* VG = nullptr, int64_t vg_floats = 0);
// tile 69 (conv_halo.hip): persistent 3x3 conv 16 -> 32 channels with the 2x2
// max pool fused, input patches staged once per 8 x 16-pixel tile
int launch_halo(const ConvArgs& a, hipStream_t st);
// tile 73 (conv_wpool.hip): the Winograd F(2x2,3x3) form of tile 69 (16 -> 32 channels, 2x2 max pool
// fused, persistent, in-register inverse transform; bit-identical to tile 61); U = po_conv_desc.Wwino
int launch_wpool(const ConvArgs& a, const float* U, hipStream_t st);

}  // namespace po
