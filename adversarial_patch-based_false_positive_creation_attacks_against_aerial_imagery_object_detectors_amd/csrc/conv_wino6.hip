// Winograd F(4x4,3x3) po_conv tile 71 (staging 16): conv_wino6_k, a
// persistent kernel on tile 70's pipeline (conv_wino5.hip) with 4x4 output
// tiles.
#pragma clang fp contract(off)
#include "conv_common.h"
#include "wino_common.h"

namespace {

// ---------------------------------------------------------------------------
// Tile 71 (staging 16): conv_wino6_k.
//
// F(2x2,3x3) executes 16 products per 4 outputs and input channel (4 per
// output); F(4x4,3x3) executes 36 per 16 (2.25 per output): 44 % fewer matrix
// cycles for the same convolution, and on gfx950 the fp32 MFMA shares its
// issue with the VALU, so the cycles saved are cycles saved.  The price is a
// 6x6 input transform (12 operations per 6-point transform, Lavin's B^T with
// the points 0, +-1, +-2, inf, products by powers of two folded into fmas),
// a larger inverse transform, and 2.25x the transformed weights per input
// channel (U = G g G^T, float64 on the host, rounded once).
//
// Unit = 32 4x4-tiles (512 output pixels) x 64 output channels x one split-K
// slice; one 512-thread workgroup per CU walks the units (tile 70's order and
// pipelining: the next unit's first input rows and B fragments are requested
// under this unit's last MFMAs).
//   * input: thread (tile tid >> 4, channel tid & 15) loads its 6x6 patch of
//     one channel (36 dword loads; rows by per-thread offsets, columns as
//     uniform steps in the scalar offset), transforms it in registers and
//     writes the 36 components to V[xi][tile][16 channels] (73,728 B, double
//     buffered: 144 KiB of LDS);
//   * GEMMs: wave w owns 32 output channels (w >> 2) and 9 of the 36
//     components (9 (w & 3) ..): one 32x32 accumulator per component (144
//     accumulator registers), 8 v_mfma_f32_32x32x2_f32 per component and
//     k-step; B fragments ride a three-deep register ring, each requested
//     three components before its use;
//   * epilogue: four passes of 8 tiles.  Each stages its 8 accumulator rows of
//     every component in LDS (M[xi][tile][64], the two 32-lane halves of a
//     wave XOR-swizzled apart), inverse-transforms one (tile, channel) per
//     thread (Y = A^T M A) into LDS, and applies tile 70's epilogue with
//     16-byte lanes (thread: one pixel of one tile x 4 channels per store).
//     Every epilogue memory operation is an unconditional buffer op, and a
//     pass's inputs are requested before the previous pass's stores (vmcnt
//     counts loads and stores in one queue), so no wait covers a store.
// Numerics: each output sums 36 transformed products per input channel; the
// transforms' coefficients (up to 5 in B^T, 8 in A^T) cost accuracy against
// F(2x2) (DESIGN.md §4 tabulates the per-layer error against float64), and
// the plan may keep any layer on tile 70.
constexpr int T6 = 32;                      // 4x4 output tiles per unit
constexpr int N6 = 64;                      // output channels per unit
constexpr int NX6 = 36;                     // transform components
constexpr int CPW6 = 9;                     // components per wave
constexpr int V6_FLOATS = NX6 * T6 * WK;    // one transformed-input buffer (73,728 B)
constexpr int TP6 = 8;                      // tiles per epilogue pass

// V[xi][tile][16 channels]: 16-byte chunk `chunk` of tile t, swizzled by tile
__device__ __forceinline__ int v6idx(int xi, int t, int chunk) {
  return (xi * T6 + t) * WK + ((chunk ^ ((t >> 2) & 3)) << 2);
}

// 1-D F(4,3) input transform r = B^T d (Lavin: rows 4 0 -5 0 1 0 / 0 -4 -4 1 1 0 /
// 0 4 -4 -1 1 0 / 0 -2 -1 2 1 0 / 0 2 -1 -2 1 0 / 0 4 0 -5 0 1)
__device__ __forceinline__ void bt6(float d0, float d1, float d2, float d3, float d4, float d5, float* r) {
  const float a = __builtin_fmaf(-4.f, d2, d4), b = __builtin_fmaf(-4.f, d1, d3);
  const float c = d4 - d2, e = d3 - d1;
  r[0] = __builtin_fmaf(4.f, d0, __builtin_fmaf(-5.f, d2, d4));
  r[1] = a + b;
  r[2] = a - b;
  r[3] = __builtin_fmaf(2.f, e, c);
  r[4] = __builtin_fmaf(-2.f, e, c);
  r[5] = __builtin_fmaf(4.f, d1, __builtin_fmaf(-5.f, d3, d5));
}
// bt6 on pairs (v_pk_fma_f32 / v_pk_add_f32): the same operations per element
__device__ __forceinline__ void bt6v(f2v d0, f2v d1, f2v d2, f2v d3, f2v d4, f2v d5, f2v* r) {
  const f2v m4 = {-4.f, -4.f}, p4 = {4.f, 4.f}, m5 = {-5.f, -5.f}, p2 = {2.f, 2.f}, m2 = {-2.f, -2.f};
  const f2v a = __builtin_elementwise_fma(m4, d2, d4), b = __builtin_elementwise_fma(m4, d1, d3);
  const f2v c = d4 - d2, e = d3 - d1;
  r[0] = __builtin_elementwise_fma(p4, d0, __builtin_elementwise_fma(m5, d2, d4));
  r[1] = a + b;
  r[2] = a - b;
  r[3] = __builtin_elementwise_fma(p2, e, c);
  r[4] = __builtin_elementwise_fma(m2, e, c);
  r[5] = __builtin_elementwise_fma(p4, d1, __builtin_elementwise_fma(m5, d3, d5));
}
// 1-D inverse y = A^T m (rows 1 1 1 1 1 0 / 0 1 -1 2 -2 0 / 0 1 1 4 4 0 / 0 1 -1 8 -8 1)
__device__ __forceinline__ void at6(float m0, float m1, float m2, float m3, float m4, float m5, float* y) {
  const float p = m1 + m2, q = m1 - m2, r = m3 + m4, s = m3 - m4;
  y[0] = (m0 + p) + r;
  y[1] = __builtin_fmaf(2.f, s, q);
  y[2] = __builtin_fmaf(4.f, r, p);
  y[3] = __builtin_fmaf(8.f, s, q) + m5;
}

// Gradient-cone boxes (ConvArgs.gbox, destination pixels [r0,r1) x [c0,c1) of
// image b): the image's GEMM rows l < h*w enumerate the 4x4 tiles meeting its
// box row-major, the rest are dead (conv_wino.hip tile_point with 4x4 tiles)
struct Box6 {
  int t0, u0, h, w;
};
__device__ __forceinline__ Box6 box6(const ConvArgs& a, int b) {
  const int4 bx = reinterpret_cast<const int4*>(a.gbox)[b];
  const int t0 = bx.x >> 2, t1 = (bx.z + 3) >> 2, u0 = bx.y >> 2, u1 = (bx.w + 3) >> 2;
  return {t0, u0, max(t1 - t0, 0), max(u1 - u0, 0)};
}
// GEMM row m -> image b, tile (ti, tj); false: the row computes nothing
__device__ __forceinline__ bool tile_pt6(const ConvArgs& a, int Ht, int Wt, int m, int& b, int& ti, int& tj) {
  if (!a.gbox) return tile_point_magic(a, Ht, Wt, m, b, ti, tj);
  const int per = Ht * Wt;
  const bool in = m < a.B * per;
  b = in ? po::div_by(m, a.mg_tiles, a.sh_tiles) : 0;
  const int l = in ? m - b * per : 0;
  const Box6 x = box6(a, b);
  const bool ok = in && l < x.h * x.w;
  const int q = ok ? l / x.w : 0;
  ti = x.t0 + q;
  tj = x.u0 + (ok ? l - q * x.w : 0);
  return ok;
}
// whether unit u (its 32 GEMM rows; wave-uniform) holds a live tile: always on
// a full map, with boxes when one of the (at most a few) images it spans has
// one of its first h*w rows in it
__device__ __forceinline__ bool unit_live6(const ConvArgs& a, int Ht, int Wt, int u, int mn) {
  if (!a.gbox) return true;
  const int per = Ht * Wt;
  const int s = po::div_by(u, a.mg_mn, a.sh_mn);
  const int tm = po::div_by(u - s * mn, a.mg_ntn, a.sh_ntn);
  const int m0 = tm * 32;
  const int b0 = po::div_by(m0, a.mg_tiles, a.sh_tiles);
  const int b1 = min(po::div_by(m0 + 31, a.mg_tiles, a.sh_tiles), a.B - 1);
  for (int b = b0; b <= b1; ++b) {
    const Box6 x = box6(a, b);
    if (max(m0 - b * per, 0) < x.h * x.w) return true;
  }
  return false;
}

#ifdef PO_W6_STAMP
// diagnostic build only (tools/w6_phases.py): per workgroup, shader cycles
// (s_memtime) summed over its units per phase -- [0] unit top through the
// k-loop, [1] the peeled last step, [2] the epilogue passes -- [3] units,
// [4]/[5] s_memrealtime at start / end
__device__ unsigned long long g_w6_stamp[1 << 12][8];
#define PO_W6_T(v) v = __builtin_amdgcn_s_memtime()
#else
#define PO_W6_T(v) do { } while (0)
#endif

#ifdef PO_W6_NOSTORE
// diagnostic build only: the epilogue's global stores removed (what the stores cost)
#define W6ST(x) do { } while (0)
#else
#define W6ST(x) x
#endif

// MODE 0: po_conv epilogue (fields EF), 1: raw split-K partials.  PT (tile 72):
// the transformed input comes from VG (wino6_pre_k) straight into registers
template <int MODE, int EF, bool PT = false>
__global__ __launch_bounds__(512, 1) void conv_wino6_k(const ConvArgs a, const float* __restrict__ U, int Ht, int Wt,
                                                       int units, int mn, const float* __restrict__ VG,
                                                       uint32_t vg_bytes) {
  __shared__ __attribute__((aligned(16))) float smem[2 * V6_FLOATS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave_u = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5;
  const int nbw = wave_u >> 2;                 // the wave's 32-channel half of the unit
  const int xq = (wave_u & 3) * CPW6;          // its first component
  const int G = gridDim.x;
  const int kc_n = a.Cin_p / WK;
  const int wpp = a.Cout_p >> 5;

  // ---- buffer resources (host: every extent < 2^31 bytes, the input < 2^30)
  const uint32_t npix = (uint32_t)a.B * (uint32_t)a.Hout * (uint32_t)a.Wout;
  const uint32_t dst_bytes = npix * (uint32_t)a.Cout_p * 4u;
  const uint32_t bits_bytes = npix * (uint32_t)wpp * 4u;
  const uint32_t pool_bytes = (npix >> 2) * (uint32_t)a.Cout_p * 4u;   // EF_POOL: [B][Hout/2][Wout/2][Cout_p] floats
  const uint32_t in_bytes = (uint32_t)__builtin_amdgcn_readfirstlane(a.in_bytes);
  const __amdgpu_buffer_rsrc_t in_rs = rsrc(a.in, in_bytes);
  __amdgpu_buffer_rsrc_t rs_out = in_rs, rs_bias = in_rs;
  if constexpr (MODE == 0) rs_out = rsrc(a.y, (EF & (EF_Y | EF_ACC)) ? dst_bytes : 0u);
  if constexpr (MODE == 1) rs_out = rsrc(a.ws, (uint32_t)a.ksplit * (uint32_t)a.M * (uint32_t)a.N * 4u);
  if constexpr (MODE == 0) rs_bias = rsrc(a.bias, a.bias ? (uint32_t)a.N * 4u : 0u);

  // ---- unit u -> (first tile row m0, n-block tn, split-K slice s, its k-steps [ks0, ks1)), wave-uniform
  auto unit = [&](int u, int& m0, int& tn, int& s, int& ks0, int& ks1) {
    s = po::div_by(u, a.mg_mn, a.sh_mn);
    const int rem = u - s * mn;
    const int tm = po::div_by(rem, a.mg_ntn, a.sh_ntn);
    tn = rem - tm * a.ntiles_n;
    m0 = tm * T6;
    ks0 = po::div_by(s * kc_n, a.mg_ks, a.sh_ks);
    ks1 = po::div_by((s + 1) * kc_n, a.mg_ks, a.sh_ks);
  };

  // ---- input staging: thread (tile r, channel c) loads its 6x6 patch of one channel.
  // Two registers per thread across the k-loop: rbase = byte offset of the
  // patch's pixel (row 1, column 1), i.e. (4 ti, 4 tj): never negative; okm =
  // row (bits 0-5) and column (bits 8-13) validity.  Row i >= 1, column j >= 1
  // read rbase + (i-1)*row_bytes + (j-1)*pix_bytes with the steps in the scalar
  // offset; row 0 / column 0 subtract row_bytes / pix_bytes in the vector
  // offset, taken only when that row / column is inside the map (so the vector
  // offset is the true, non-negative one: no reliance on 32-bit wrap-around)
  const int r = tid >> 4, c = tid & 15;
  const uint32_t pix_bytes = (uint32_t)a.Cin_p * 4u;
  const uint32_t row_bytes = (uint32_t)a.Win * pix_bytes;
  uint32_t rbase = 0u, okm = 0u;
  auto offsets = [&](int m0) {
    int b, ti, tj;
    const bool ok_t = tile_pt6(a, Ht, Wt, m0 + r, b, ti, tj);
    const int y0 = 4 * ti - 1, x0 = 4 * tj - 1;
    rbase = (((uint32_t)b * a.Hin + (uint32_t)(4 * ti)) * a.Win + (uint32_t)(4 * tj)) * pix_bytes + 4u * c;
    okm = 0u;
#pragma unroll
    for (int i = 0; i < 6; ++i) okm |= (ok_t && (unsigned)(y0 + i) < (unsigned)a.Hin ? 1u : 0u) << i;
#pragma unroll
    for (int j = 0; j < 6; ++j) okm |= ((unsigned)(x0 + j) < (unsigned)a.Win ? 1u : 0u) << (8 + j);
  };
  f2v d[18];                                   // d[3 i + jp] = patch row i, columns 2jp, 2jp+1
  // row i of step ks's patches into d (6 loads; opaque per call: hoisted out of
  // the k-loop, the per-load selects would hold 36 registers across it).
  // Branch-free: a wave-uniform fast path for tiles inside the map's columns
  // made the compiler's vmcnt waits after the merge count every row load.
  auto grow = [&](int ks, int i) {
    const uint32_t cb = (uint32_t)__builtin_amdgcn_readfirstlane(ks * (WK * 4));
    uint32_t rb = rbase, om = okm;
    asm volatile("" : "+v"(rb), "+v"(om));
    const bool rok = (om >> i) & 1u;
    const uint32_t rr = i == 0 ? rb - row_bytes : rb;
    const uint32_t rv = rok ? rr : kOOB;                                  // columns 1..5
    const uint32_t rv0 = (rok && ((om >> 8) & 1u)) ? rr - pix_bytes : kOOB;  // column 0
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const uint32_t vo = j == 0 ? rv0 : (((om >> (8 + j)) & 1u) ? rv : kOOB);
      const uint32_t so = cb + (i == 0 ? 0u : (uint32_t)(i - 1) * row_bytes) + (j == 0 ? 0u : (uint32_t)(j - 1) * pix_bytes);
      d[3 * i + (j >> 1)][j & 1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(in_rs, vo, so, 0));
    }
  };
  auto gload = [&](int ks) {
#pragma unroll
    for (int i = 0; i < 6; ++i) grow(ks, i);
  };
  // V = B^T d B on column pairs / row pairs (packed f32): the columns (pairs of
  // columns), a 2x2 transposition of every block, then the rows (pairs of rows);
  // component xi = 6 i + j.  The same operations as bt6 lane by lane.
  auto transform = [&](float* Vb) {
#ifdef PO_W6_ABL_NOVWRITE
    return;                                    // diagnostic only (wrong results): no transform, no V writes
#endif
#ifdef PO_W6_ABL_NOTRANS
    // diagnostic only (wrong results): the raw rows written as they are, no transform VALU
    {
      float* dst = Vb + v6idx(0, r, c >> 2) + (c & 3);
#pragma unroll
      for (int xi = 0; xi < 36; ++xi) dst[xi * T6 * WK] = d[xi >> 1][xi & 1];
      return;
    }
#endif
    f2v t[6][3];                               // t[i][jp]: (B^T d)[i][2jp], [i][2jp+1]
#pragma unroll
    for (int jp = 0; jp < 3; ++jp) {
      f2v col[6];
      bt6v(d[jp], d[3 + jp], d[6 + jp], d[9 + jp], d[12 + jp], d[15 + jp], col);
#pragma unroll
      for (int i = 0; i < 6; ++i) t[i][jp] = col[i];
      __builtin_amdgcn_sched_barrier(0);     // one column pair at a time: d's registers turn into t's
    }
    float* dst = Vb + v6idx(0, r, c >> 2) + (c & 3);
#pragma unroll
    for (int ip = 0; ip < 3; ++ip) {
      f2v rw[6];                               // (t[2ip][j], t[2ip+1][j])
#pragma unroll
      for (int j = 0; j < 6; ++j) rw[j] = f2v{t[2 * ip][j >> 1][j & 1], t[2 * ip + 1][j >> 1][j & 1]};
      f2v e[6];
      bt6v(rw[0], rw[1], rw[2], rw[3], rw[4], rw[5], e);
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        dst[(6 * (2 * ip) + j) * T6 * WK] = e[j][0];     // v6idx(xi, r, .) = v6idx(0, r, .) + xi*T6*WK
        dst[(6 * (2 * ip + 1) + j) * T6 * WK] = e[j][1];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- B operand: fragment-ordered U [N/32][Cin_p/16][36][2][64][4] through a buffer
  // resource (per-lane 16-byte offset, block offset in a scalar register)
  const __amdgpu_buffer_rsrc_t u_rs = rsrc(U, (uint32_t)a.N * (uint32_t)NX6 * (uint32_t)a.Cin_p * 4u);
  const uint32_t u_lane = (uint32_t)lane * 16u;
  float4 bq[3][2];
  auto bload = [&](int slot, int cc, int ks, int tnn) {
#ifdef PO_W6_ABL_UHOT
    // diagnostic only (wrong results): every B fragment from one block, always cache-hot
    const uint32_t blk = (uint32_t)__builtin_amdgcn_readfirstlane((nbw * NX6 + xq + cc) * 512 * 4) * 0u;
#else
    const uint32_t blk = (uint32_t)__builtin_amdgcn_readfirstlane(
        ((((2 * tnn + nbw) * kc_n + ks) * NX6 + xq + cc) * 512) * 4);
#endif
    bq[slot][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(u_rs, u_lane, blk, 0));
    bq[slot][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(u_rs, u_lane + 1024u, blk, 0));
  };
  // ---- A operand (tile 72): VG [m-block][k-step][36][32 tiles][16 channels]; lane
  // (tile lane & 31, half h) takes channels 8h .. 8h+7 of its tile (two 16-byte
  // loads, a wave's 2 KB contiguous), on a ring beside the B fragments'
  const __amdgpu_buffer_rsrc_t v_rs = rsrc(VG, PT ? vg_bytes : 0u);
  const uint32_t a_lane = ((uint32_t)(lane & 31) * WK + 8u * (uint32_t)h) * 4u;
  float4 aq[3][2];
  auto aload = [&](int slot, int cc, int ks, int tmm) {
    const uint32_t blk = (uint32_t)__builtin_amdgcn_readfirstlane(((tmm * kc_n + ks) * NX6 + xq + cc) * (T6 * WK * 4));
    aq[slot][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(v_rs, a_lane, blk, 0));
    aq[slot][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(v_rs, a_lane + 16u, blk, 0));
  };
  floatx16 acc[CPW6];
  // the wave's 9 components of one k-step: component cc's MFMAs, each half's A
  // fragment of component cc + 1 read from LDS as soon as its registers are
  // free (after the 4 MFMAs that use them), and the ring slot cc frees refilled
  // with component cc + 3 (this k-step) or cc - 6 (the next; not on the last step)
  // !last: row cc of step kg's input patches requested after component cc's
  // MFMAs (cc < 6), so the row loads issue beside the matrix work
  auto comps = [&](const float* Vb, int ks, int tnn, int tmm, auto last_c, int kg) {
    constexpr bool last = decltype(last_c)::value;
    const int o0 = v6idx(xq, lane & 31, 2 * h), o1 = o0 ^ 4;     // chunks 2h, 2h + 1: swizzled apart in bit 0
    float4 a0, a1;
    if constexpr (!PT) {
      a0 = *reinterpret_cast<const float4*>(Vb + o0);
      a1 = *reinterpret_cast<const float4*>(Vb + o1);
    }
#pragma unroll
    for (int cc = 0; cc < CPW6; ++cc) {
      if constexpr (PT) {
        a0 = aq[cc % 3][0];
        a1 = aq[cc % 3][1];
      }
      const float4 b0 = bq[cc % 3][0], b1 = bq[cc % 3][1];
      acc[cc] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, b0.x, acc[cc], 0, 0, 0);   // step s <-> channel 8h + s
      acc[cc] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, b0.y, acc[cc], 0, 0, 0);
      acc[cc] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.z, b0.z, acc[cc], 0, 0, 0);
      acc[cc] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.w, b0.w, acc[cc], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (!PT && cc + 1 < CPW6) a0 = *reinterpret_cast<const float4*>(Vb + o0 + (cc + 1) * T6 * WK);
      __builtin_amdgcn_sched_barrier(0);
      acc[cc] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.x, b1.x, acc[cc], 0, 0, 0);
      acc[cc] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.y, b1.y, acc[cc], 0, 0, 0);
      acc[cc] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.z, b1.z, acc[cc], 0, 0, 0);
      acc[cc] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.w, b1.w, acc[cc], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (!PT && cc + 1 < CPW6) a1 = *reinterpret_cast<const float4*>(Vb + o1 + (cc + 1) * T6 * WK);
      if (cc + 3 < CPW6) {
        bload(cc % 3, cc + 3, ks, tnn);
        if constexpr (PT) aload(cc % 3, cc + 3, ks, tmm);
      } else if (!last) {
        bload(cc % 3, cc - 6, ks + 1, tnn);
        if constexpr (PT) aload(cc % 3, cc - 6, ks + 1, tmm);
      }
      if (!PT && cc < 6 && !last) grow(kg, cc);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- the unit loop
  int u = po::xcd_remap();                     // host: gridDim.x <= units
  while (u < units && !unit_live6(a, Ht, Wt, u, mn)) u += G;       // boxed: skip units with no live tile
  if (u >= units) return;                      // (uniform: every wave of the workgroup leaves)
  int m0, tn, s, ks0, ks1;
  unit(u, m0, tn, s, ks0, ks1);
  if constexpr (!PT) {
    offsets(m0);
    gload(ks0);
  }
  float* const M = smem;
  // ---- epilogue state.  The epilogue runs in four passes of 8 tiles; passes 0
  // and 1 emit at once, passes 2 and 3 leave their outputs in LDS (the V1 buffer,
  // free until the next unit's first k-step ends) and emit after the next
  // unit's first transform, so their stores drain under its first MFMAs.
  const int n_loc = 4 * (tid & 15);            // the emitting thread's 4 channels in the unit
  const int epx = (tid >> 4) & 15;             // its pixel of a tile: row epx >> 2, column epx & 3
  const int et = tid >> 8;                     // its tiles of a pass: et, et + 2, et + 4, et + 6
  constexpr bool RES = MODE == 0 && (EF & EF_RES), ACC = MODE == 0 && (EF & EF_ACC);
  constexpr bool MB = MODE == 0 && (EF & EF_MB), Y2 = MODE == 0 && (EF & EF_Y2);
  // POOL: a 4x4 output tile holds four 2x2 pool windows; in the passes a thread
  // owns window pw = (tid >> 4) & 3 of tile pt = tid >> 6 for the 4 channels n_loc
  constexpr bool POOL = MODE == 0 && (EF & EF_POOL);
  const int pw = (tid >> 4) & 3, pt = tid >> 6;
  int n4 = 0, es = 0;                          // the staged unit's channel base and split-K slice
  float4 bias4 = make_float4(0.f, 0.f, 0.f, 0.f);
  // per pass parity: pixels (MODE 1: workspace rows) of the thread's four tiles,
  // their output mask (0: nothing staged yet), and the epilogue inputs
  uint32_t epix[2][4], eok[2] = {0u, 0u};
  float4 pin[2][4];
  uint32_t pm[2][4], pm2[2][4];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      epix[q][k] = pm[q][k] = pm2[q][k] = 0u;
      pin[q][k] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  int cur_m0 = 0;
  auto inputs = [&](int p) {
    const int q = p & 1;
    eok[q] = 0u;
    if constexpr (POOL) {
      // the window's pooled pixel (full even maps, no boxes: host checks)
      int b, ti, tj;
      const bool tl = tile_pt6(a, Ht, Wt, cur_m0 + TP6 * p + pt, b, ti, tj);
      const int pi = 2 * ti + (pw >> 1), pj = 2 * tj + (pw & 1);
      const bool ok = tl && pi < (a.Hout >> 1) && pj < (a.Wout >> 1);
      eok[q] = ok ? 1u : 0u;
      epix[q][0] = ((uint32_t)b * (uint32_t)(a.Hout >> 1) + pi) * (uint32_t)(a.Wout >> 1) + pj;
      return;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      int b, ti, tj;
      const bool tl = tile_pt6(a, Ht, Wt, cur_m0 + TP6 * p + et + 2 * k, b, ti, tj);
      const int i = 4 * ti + (epx >> 2), j = 4 * tj + (epx & 3);
      bool ok = tl && i < a.Hout && j < a.Wout;
      // split-K partials at conv_reduce_k's GEMM rows: row-major over the map,
      // or over the image's box (conv_common.h grid_point)
      int wl = i * a.Wg + j;
      if (a.gbox) {                                // only the box's pixels are written
        const int4 bx = reinterpret_cast<const int4*>(a.gbox)[b];
        ok = ok && i >= bx.x && i < bx.z && j >= bx.y && j < bx.w;
        if constexpr (MODE == 1) {
          const int i0 = max(bx.x, 0), j0 = max(bx.y, 0);
          wl = (i - i0) * (min(bx.w, a.Wg) - j0) + j - j0;
        }
      }
      eok[q] |= (ok ? 1u : 0u) << k;
      epix[q][k] = MODE == 1 ? (uint32_t)b * a.mrows + (uint32_t)wl : ((uint32_t)b * a.Hout + i) * a.Wout + j;
      const uint32_t o = (epix[q][k] * (uint32_t)a.Cout_p + n4) * 4u;
      const uint32_t wo = (epix[q][k] * (uint32_t)wpp + (uint32_t)(n4 >> 5)) * 4u;
      if constexpr (RES) pin[q][k] = bld4(rsrc(a.res, dst_bytes), ok ? o : kOOB);
      if constexpr (ACC) pin[q][k] = bld4(rs_out, ok ? o : kOOB);
      if constexpr (MB) pm[q][k] = bld1(rsrc(a.mbits, bits_bytes), ok ? wo : kOOB);
      if constexpr (Y2) pm2[q][k] = bld1(rsrc(a.m2bits, bits_bytes), ok ? wo : kOOB);
    }
  };
  // outputs of pass p of the staged unit from its LDS slot (every store
  // unconditional: a masked one goes out of range)
  auto emit = [&](int p) {
    const int q = p & 1;
    if constexpr (POOL) {
      // window pw of tile pt: its pixels (2wy + dy, 2wx + dx), position k = 2dy + dx,
      // bias + activation per pixel, then po_maxpool2_fwd's rule (first position on
      // ties, NaN wins) and the slope-carrying argmax codes (conv_pool_epilogue)
      int rrow = V6_FLOATS + q * (TP6 * 16 * N6) + (pt * 16 + 8 * (pw >> 1) + 2 * (pw & 1)) * N6 + n_loc;
      asm volatile("" : "+v"(rrow));
      float pv[4] = {0.f, 0.f, 0.f, 0.f};
      uint32_t arg[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float4 v = *reinterpret_cast<const float4*>(smem + rrow + (4 * (k >> 1) + (k & 1)) * N6);
        const float xv[4] = {v.x + bias4.x, v.y + bias4.y, v.z + bias4.z, v.w + bias4.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float x = po::leaky_or_id(xv[c], po::act_slope(a.act));
          if (k == 0 || x > pv[c] || isnan(x)) { pv[c] = x; arg[c] = (uint32_t)k; }
        }
      }
      uint32_t code = 0u;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (a.act) arg[c] |= 8u | (pv[c] > 0.f ? 0u : 4u);
        code |= arg[c] << (8 * c);
      }
      const bool ok = eok[q] & 1u;
      const uint32_t po = epix[q][0] * (uint32_t)a.Cout_p + n4;      // pooled element (< 2^31: host check)
      W6ST(bst4(make_float4(pv[0], pv[1], pv[2], pv[3]), rsrc(a.pool_y, pool_bytes), ok ? po * 4u : kOOB));
      W6ST(bst1(code, rsrc(a.pool_am, pool_bytes >> 2), ok ? po : kOOB));
      return;
    }
    int rrow = V6_FLOATS + q * (TP6 * 16 * N6) + (et * 16 + epx) * N6 + n_loc;
    asm volatile("" : "+v"(rrow));
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 v = *reinterpret_cast<const float4*>(smem + rrow + 2 * k * 16 * N6);
      const bool ok = (eok[q] >> k) & 1u;
      const uint32_t pix = epix[q][k];
      if constexpr (MODE == 1) {
        const uint32_t o = (((uint32_t)es * (uint32_t)a.M + pix) * (uint32_t)a.N + n4) * 4u;
        W6ST(bst4(v, rs_out, ok ? o : kOOB));
      } else {
        const uint32_t o = (pix * (uint32_t)a.Cout_p + n4) * 4u;
        float x[4] = {v.x + bias4.x, v.y + bias4.y, v.z + bias4.z, v.w + bias4.w};
#pragma unroll
        for (int cch = 0; cch < 4; ++cch) x[cch] = po::leaky_or_id(x[cch], po::act_slope(a.act));
        if constexpr (ACC) {
          x[0] += pin[q][k].x; x[1] += pin[q][k].y; x[2] += pin[q][k].z; x[3] += pin[q][k].w;
        }
        float4 out = make_float4(x[0], x[1], x[2], x[3]);
        if constexpr (MB) {
          const float4 g = po::leaky_grad_bits(pm[q][k], n4);
          out = make_float4(x[0] * g.x, x[1] * g.y, x[2] * g.z, x[3] * g.w);
        }
        if constexpr ((EF & EF_Y) != 0) W6ST(bst4(out, rs_out, ok ? o : kOOB));
        if constexpr (RES) {
          const float4 rr = pin[q][k];
          W6ST(bst4(make_float4(x[0] + rr.x, x[1] + rr.y, x[2] + rr.z, x[3] + rr.w), rsrc(a.sum, dst_bytes), ok ? o : kOOB));
        }
        if constexpr (Y2) {
          const float4 g2 = po::leaky_grad_bits(pm2[q][k], n4);
          W6ST(bst4(make_float4(x[0] * g2.x, x[1] * g2.y, x[2] * g2.z, x[3] * g2.w), rsrc(a.y2, dst_bytes), ok ? o : kOOB));
        }
        if constexpr ((EF & EF_YB) != 0) {
          // sign bits: 8 lanes hold the 32 channels of one word (DPP row shifts, tile 70)
          const uint32_t nib = ((out.x > 0.f ? 1u : 0u) | (out.y > 0.f ? 2u : 0u) | (out.z > 0.f ? 4u : 0u) |
                                (out.w > 0.f ? 8u : 0u)) & (0u - (uint32_t)ok);
          uint32_t w = nib << (4 * (lane & 7));
          w |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x101, 0xF, 0xF, false);   // row_shl:1
          w |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x102, 0xF, 0xF, false);   // row_shl:2
          w |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x104, 0xF, 0xF, false);   // row_shl:4
          W6ST(bst1(w, rsrc(a.ybits, bits_bytes),
                    (ok && (lane & 7) == 0) ? (pix * (uint32_t)wpp + (uint32_t)(n4 >> 5)) * 4u : kOOB));
        }
      }
    }
  };
#ifdef PO_W6_STAMP
  unsigned long long ph[3] = {0, 0, 0}, t0 = 0, t1 = 0, t2 = 0, t3 = 0, nunits = 0;
  const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  for (;;) {
    PO_W6_T(t0);
    __syncthreads();                           // the previous unit's LDS traffic is done
    int ks = ks0;
    if constexpr (PT) {
      // tile 72: the unit's first A and B fragments, then the previous unit's
      // last two passes (their stores behind the loads), then the k-steps --
      // each wave on its own: no LDS and no barrier until the epilogue
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) {
        aload(cc, cc, ks0, m0 / T6);
        bload(cc, cc, ks0, tn);
      }
      __builtin_amdgcn_sched_barrier(0);
      emit(2);
      emit(3);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int cc = 0; cc < CPW6; ++cc)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[cc][e] = 0.f;
      do {                                     // steps ks0 .. ks1-2
        comps(smem, ks, tn, m0 / T6, std::false_type{}, 0);
      } while (++ks < ks1 - 1);
    } else {
      transform(smem);                         // step ks0 into V0
      __builtin_amdgcn_sched_barrier(0);
      emit(2);                                 // the previous unit's last two passes (masked on the first)
      emit(3);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int cc = 0; cc < CPW6; ++cc)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[cc][e] = 0.f;
      gload(ks0 + 1);                          // host: ks1 - ks0 >= 2
      // the first B fragments after the rows, as around the loop (the compiler's
      // vmcnt waits at the loop head then count the fragments as later than the rows)
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) bload(cc, cc, ks0, tn);
      __syncthreads();
      // every wave: the next step's transform (its rows requested during this
      // unit's previous step, or above), then this step's MFMAs with the rows of
      // the step after requested between them -- the 36 row loads of a k-step
      // issued beside the matrix work rather than in a burst that the whole
      // workgroup waits for at the barrier.  (The fp32 MFMA does not co-issue
      // with the VALU, so a SIMD's time is the sum in any order.  Staggering the
      // two waves of a SIMD as tile 70 does -- waves 4-7 transforming before their
      // MFMAs -- measured 7 % slower per k-step here.)
      do {                                     // steps ks0 .. ks1-2
        const float* Vc = smem + ((ks - ks0) & 1) * V6_FLOATS;
        float* Vn = smem + (((ks - ks0) & 1) ^ 1) * V6_FLOATS;
        const int k2 = min(ks + 2, ks1 - 1);
        transform(Vn);
        __builtin_amdgcn_sched_barrier(0);
        comps(Vc, ks, tn, 0, std::false_type{}, k2);
#ifndef PO_W6_ABL_NOBAR
        __syncthreads();
#endif
      } while (++ks < ks1 - 1);
    }
    // ---- the last step, peeled (no prefetch past the unit)
    PO_W6_T(t1);
    const float* Vl = smem + ((ks - ks0) & 1) * V6_FLOATS;
    cur_m0 = m0;
    const int cur_tn = tn, cur_s = s;
    int nu = u + G;
    while (nu < units && !unit_live6(a, Ht, Wt, nu, mn)) nu += G;
    const bool more = nu < units;
    unit(more ? nu : u, m0, tn, s, ks0, ks1);
    comps(Vl, ks, cur_tn, cur_m0 / T6, std::true_type{}, 0);

    // ---- epilogue: four passes of 8 tiles
    PO_W6_T(t2);
    n4 = cur_tn * N6 + n_loc;
    es = cur_s;
    if constexpr (MODE == 0) bias4 = bld4(rs_bias, (uint32_t)n4 * 4u);
    inputs(0);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      __syncthreads();                         // the k-loop's / previous pass's LDS reads are done
      {
        // stage rows e = 4p .. 4p+3 of the wave's accumulators: row (e & 3) + 4h of the pass
        // (column n of the unit's 64, the wave halves XOR-swizzled by 32 apart)
        int wrow = 4 * h * N6 + ((32 * nbw + (lane & 31)) ^ (32 * h));
        asm volatile("" : "+v"(wrow));
#pragma unroll
        for (int cc = 0; cc < CPW6; ++cc)
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4) M[((xq + cc) * TP6 + e4) * N6 + wrow] = acc[cc][4 * p + e4];
      }
      __syncthreads();
      {
        // inverse transform: thread (tile wave, channel lane) of the pass, into LDS slot p & 1
        int rd = wave_u * N6 + (lane ^ (32 * ((wave_u >> 2) & 1)));
        asm volatile("" : "+v"(rd));
        float z[6][4];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          float m[6];
#pragma unroll
          for (int j = 0; j < 6; ++j) m[j] = M[(6 * i + j) * TP6 * N6 + rd];
          at6(m[0], m[1], m[2], m[3], m[4], m[5], z[i]);
        }
        int wr = V6_FLOATS + (p & 1) * (TP6 * 16 * N6) + wave_u * 16 * N6 + lane;
        asm volatile("" : "+v"(wr));
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          float y[4];
          at6(z[0][jj], z[1][jj], z[2][jj], z[3][jj], z[4][jj], z[5][jj], y);
#pragma unroll
          for (int ii = 0; ii < 4; ++ii) smem[wr + (4 * ii + jj) * N6] = y[ii];
        }
      }
      if (p < 3) inputs(p + 1);                // requested before this pass's stores
      if (p < 2) {
        __syncthreads();
        emit(p);
      }
      if (!PT && p == 1) {
        // the next unit's first input rows and B fragments (the last unit re-reads
        // its own: branch-free), requested halfway through the epilogue: earlier,
        // their 60 registers would sit beside the accumulators of passes 1-3
        offsets(m0);
        gload(ks0);
      }
    }
    PO_W6_T(t3);
#ifdef PO_W6_STAMP
    ph[0] += t1 - t0;
    ph[1] += t2 - t1;
    ph[2] += t3 - t2;
    ++nunits;
#endif
    if (!more) break;
    u = nu;
  }
  __syncthreads();                             // the last unit's passes 2 and 3
  emit(2);
  emit(3);
#ifdef PO_W6_STAMP
  if (tid == 0 && blockIdx.x < (1 << 12)) {
    for (int i = 0; i < 3; ++i) g_w6_stamp[blockIdx.x][i] = ph[i];
    g_w6_stamp[blockIdx.x][3] = nunits;
    g_w6_stamp[blockIdx.x][4] = rt0;
    g_w6_stamp[blockIdx.x][5] = __builtin_amdgcn_s_memrealtime();
  }
#endif
}

// ---------------------------------------------------------------------------
// Tile 72 (staging 17): the input transform as its own pass.  wino6_pre_k writes
// V = B^T d B of every 32-tile m-block and 16-channel k-step once,
// VG[m-block][k-step][xi][tile][channel] (73,728 B per block and step, the
// order conv_wino6_k<.., PT> reads A fragments in), and the GEMM kernel then
// streams its A fragments from it like its B fragments: its k-loop is MFMAs and
// 16-byte loads, with no gathers, no transform VALU, no LDS and no barrier.
// The price is VG's round trip through HBM (2.25 x the input for interior
// 4x4 tiles): the plan's tuner weighs it per launch against tile 71.
// Block (m-block, 4 k-steps), thread (tile r, channel quad q): tile 71's
// gather (16-byte loads: a tile's 64 channels are 256 contiguous bytes) and
// transform on 4 channels at once, the components stored as 16-byte runs.
// Channels past Cin_p (Cin_p % 64 != 0) are neither read nor written.  An
// m-block without a live tile (boxes) is skipped: no unit reads it.
constexpr int PRE_KS = 4;                      // k-steps per wino6_pre_k block
__global__ __launch_bounds__(512) void wino6_pre_k(const ConvArgs a, float* __restrict__ VG, int Ht, int Wt, int xr) {
  // xr: the (m-block, k-group) blocks in an XCD-aware order -- consecutive
  // m-blocks of one k-group on one XCD, so the window rows that vertically
  // neighbouring tile rows share meet in that XCD's L2 (a bijection over the
  // grid; blocks are dispatched to the 8 XCDs round-robin in linear order)
  int bx = blockIdx.x, by = blockIdx.y;
  if (xr) {
    const int gx = gridDim.x, n = gx * gridDim.y, lin = by * gx + bx;
    const int qn = n / 8, r8 = n % 8, xcd = lin % 8;
    const int lr = (xcd < r8 ? xcd * (qn + 1) : r8 * (qn + 1) + (xcd - r8) * qn) + lin / 8;
    bx = lr % gx;
    by = lr / gx;
  }
  const int tm = bx, kc_n = a.Cin_p / WK;
  const int tid = threadIdx.x, r = tid >> 4, q = tid & 15;
  const int ks = by * PRE_KS + (q >> 2);
  if (a.gbox) {
    const int per = Ht * Wt, m0 = tm * T6;
    const int b0 = po::div_by(m0, a.mg_tiles, a.sh_tiles);
    const int b1 = min(po::div_by(m0 + T6 - 1, a.mg_tiles, a.sh_tiles), a.B - 1);
    bool live = false;
    for (int b = b0; b <= b1; ++b) {
      const Box6 x = box6(a, b);
      live = live || max(m0 - b * per, 0) < x.h * x.w;
    }
    if (!live) return;
  }
  int b, ti, tj;
  const bool ok_t = tile_pt6(a, Ht, Wt, tm * T6 + r, b, ti, tj) && ks < kc_n;
  const __amdgpu_buffer_rsrc_t in_rs = rsrc(a.in, a.in_bytes);
  const uint32_t pix_bytes = (uint32_t)a.Cin_p * 4u;
  const uint32_t base = (((uint32_t)b * a.Hin) * a.Win) * pix_bytes + (uint32_t)(ks * WK + 4 * (q & 3)) * 4u;
  float4 d[6][6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int y = 4 * ti - 1 + i;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int x = 4 * tj - 1 + j;
      const bool ok = ok_t && (unsigned)y < (unsigned)a.Hin && (unsigned)x < (unsigned)a.Win;
      const uint32_t vo = ok ? base + ((uint32_t)y * a.Win + (uint32_t)x) * pix_bytes : kOOB;
      d[i][j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(in_rs, vo, 0, 0));
    }
  }
  if (!(ks < kc_n)) return;
  // per channel: the columns, then the rows -- bt6 in tile 71's order (its
  // packed pairs compute each element with the same operations)
  float* dst = VG + ((size_t)tm * kc_n + ks) * (NX6 * T6 * WK) + r * WK + 4 * (q & 3);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float t[6][6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      float col[6];
      bt6(d[0][j][e], d[1][j][e], d[2][j][e], d[3][j][e], d[4][j][e], d[5][j][e], col);
#pragma unroll
      for (int i = 0; i < 6; ++i) t[i][j] = col[i];
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      float row[6];
      bt6(t[i][0], t[i][1], t[i][2], t[i][3], t[i][4], t[i][5], row);
#pragma unroll
      for (int j = 0; j < 6; ++j) d[i][j][e] = row[j];       // d now holds V[6i + j] for channel e
    }
  }
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) *reinterpret_cast<float4*>(dst + (6 * i + j) * T6 * WK) = d[i][j];
}
}  // namespace

namespace po {
// po_conv tile staging 16 (tile 71): conv_wino6_k, Winograd F(4x4,3x3) as a
// persistent kernel (see above).
// staging 17 (tile 72, VG != nullptr): the same GEMM and epilogues on the
// input transformed beforehand by wino6_pre_k into VG (vg_floats floats).
int launch_wino6(const ConvArgs& a, const float* U6, hipStream_t st, float* VG, int64_t vg_floats) {
  PO_REQUIRE(U6, "po_conv: tile 71 needs the F(4x4,3x3) weights (Wwino6)");
  PO_REQUIRE(a.prec == 0 && a.ntaps == 9 && a.tkw == 3 && (a.sdh == 1 || a.sdh == -1) && (a.sdw == 1 || a.sdw == -1) &&
                 a.dh0 == -a.sdh && a.dw0 == -a.sdw,
             "po_conv: Winograd tile needs a full 3x3 neighbourhood of taps");
  PO_REQUIRE(a.in_step == 1 && a.out_step == 1 && a.out_oy == 0 && a.out_ox == 0 && !a.in_org && !a.out_org,
             "po_conv: tile 71 needs stride 1 on full maps");
  PO_REQUIRE(!a.gbox || a.mrows == a.Hg * a.Wg, "po_conv: tile 71 takes gradient-cone boxes on the full grid only");
  PO_REQUIRE(a.Hg == a.Hout && a.Wg == a.Wout && a.Hin == a.Hout && a.Win == a.Wout,
             "po_conv: Winograd tile needs source, grid and destination of one size");
  PO_REQUIRE(!a.pool_y || (a.pool_am && a.ksplit == 1 && !a.gbox && a.Hout % 2 == 0 && a.Wout % 2 == 0 && !a.y &&
                           !a.res && !a.accumulate && !a.mbits && !a.y2 && !a.ybits),
             "po_conv: tile 71 fuses a pool only into a plain full-map forward (even map, no split-K, only the pooled "
             "outputs)");
  PO_REQUIRE(a.N % N6 == 0 && a.Cin_p % WK == 0, "po_conv: tile 71 needs N %% 64 == 0 and Cin_p %% 16 == 0");
  PO_REQUIRE(a.Cin_p / WK >= 2 * a.ksplit, "po_conv: tile 71 needs at least two k-steps per slice");
  PO_REQUIRE(a.ksplit == 1 || (a.ws && (int64_t)a.ksplit * a.M * a.N * 4 < (1LL << 31)),
             "po_conv: tile 71 split-K needs a workspace of < 2^31 bytes");
  PO_REQUIRE(!a.mask && !a.mask2 && !a.y_amax && !a.sum_amax && !a.y2_amax,
             "po_conv: tile 71 takes leaky masks as sign bits and no max|x| slots");
  PO_REQUIRE(!(a.res && a.accumulate), "po_conv: tile 71 does not accumulate a shortcut launch");
  PO_REQUIRE(a.in_bytes < (1u << 30), "po_conv: tile 71 needs an input of < 2^30 bytes");
  PO_REQUIRE((int64_t)a.N * NX6 * a.Cin_p * 4 < (1LL << 31), "po_conv: tile 71 weights too large");
  PO_REQUIRE((int64_t)a.B * a.Hout * a.Wout * a.Cout_p * 4 < (1LL << 31),
             "po_conv: tile 71 addresses the destination with 32-bit byte offsets (< 2^31 bytes)");
  const int Ht = (a.Hout + 3) / 4, Wt = (a.Wout + 3) / 4;
  ConvArgs b = a;
  b.ntiles_n = a.N / N6;
  div_magic(Ht * Wt, b.mg_tiles, b.sh_tiles);
  div_magic(Wt, b.mg_wt, b.sh_wt);
  const int ntm = ceil_div((int64_t)a.B * Ht * Wt, T6);
  const int mn = ntm * b.ntiles_n;
  div_magic(mn, b.mg_mn, b.sh_mn);
  div_magic(b.ntiles_n, b.mg_ntn, b.sh_ntn);
  div_magic(a.ksplit, b.mg_ks, b.sh_ks);
  PO_REQUIRE((int64_t)mn * a.ksplit < (1LL << 31), "po_conv: too many tiles");
  const int units = mn * a.ksplit;
  const int kc_n = a.Cin_p / WK;
  const int64_t vg_need = (int64_t)ntm * kc_n * NX6 * T6 * WK;
  if (VG) {
    PO_REQUIRE(vg_floats >= vg_need, "po_conv: tile 72 needs a transformed-input workspace of %lld floats (have %lld)",
               (long long)vg_need, (long long)vg_floats);
    PO_REQUIRE(vg_need * 4 < (1LL << 31), "po_conv: tile 72 transformed input must be < 2^31 bytes");
  }
  const uint32_t vg_bytes = VG ? (uint32_t)(vg_need * 4) : 0u;
  const int ef = (a.y ? EF_Y : 0) | (a.res ? EF_RES : 0) | (a.accumulate ? EF_ACC : 0) | (a.mbits ? EF_MB : 0) |
                 (a.y2 ? EF_Y2 : 0) | (a.ybits ? EF_YB : 0) | (a.pool_y ? EF_POOL : 0);
  const void* k = nullptr;
  // the epilogue-field combinations po_conv launches on full-map Winograd tiles
#define PO_W6(MODE, EF)                                                                              \
  case (MODE) * 128 + (EF):                                                                          \
    k = VG ? reinterpret_cast<const void*>(conv_wino6_k<MODE, EF, true>)                            \
           : reinterpret_cast<const void*>(conv_wino6_k<MODE, EF, false>);                          \
    break;
  const int which = a.ksplit > 1 ? 128 : ef;
  switch (which) {
    PO_W6(1, 0)
    PO_W6(0, EF_Y)
    PO_W6(0, EF_Y | EF_YB)
    PO_W6(0, EF_RES | EF_YB)
    PO_W6(0, EF_Y | EF_RES)
    PO_W6(0, EF_Y | EF_RES | EF_YB)
    PO_W6(0, EF_Y | EF_ACC)
    PO_W6(0, EF_Y | EF_MB)
    PO_W6(0, EF_Y | EF_ACC | EF_MB)
    PO_W6(0, EF_Y | EF_Y2)
    PO_W6(0, EF_Y | EF_ACC | EF_Y2)
    PO_W6(0, EF_Y | EF_MB | EF_Y2)
    PO_W6(0, EF_Y | EF_ACC | EF_MB | EF_Y2)
    PO_W6(0, EF_POOL)
    default:
      break;
  }
#undef PO_W6
  PO_REQUIRE(k, "po_conv: tile 71 has no kernel for epilogue fields 0x%x", which);
  if (VG) {
    static const int xr = [] {
      const char* e = getenv("ADVPATCH_PRE_XCD");
      return (e && e[0] == '0') ? 0 : 1;
    }();
    hipLaunchKernelGGL(wino6_pre_k, dim3(ntm, ceil_div(kc_n, PRE_KS)), dim3(512), 0, st, b, VG, Ht, Wt, xr);
    const int rc = check_launch("po_conv (tile 72 input transform)");
    if (rc) return rc;
  }
  const int resident = resident_groups_cached(k, 512);
  const int grid = units < resident ? units : resident;
  const float* vgc = VG;
  void* args[] = {&b, const_cast<float**>(&U6), const_cast<int*>(&Ht), const_cast<int*>(&Wt),
                  const_cast<int*>(&units), const_cast<int*>(&mn), const_cast<float**>(&vgc),
                  const_cast<uint32_t*>(&vg_bytes)};
  PO_REQUIRE(hipLaunchKernel(k, dim3(grid), dim3(512), args, 0, st) == hipSuccess, "po_conv: tile 71 launch failed");
  return check_launch("po_conv (winograd F(4x4) persistent)");
}
#ifdef PO_W6_STAMP
extern "C" int po_debug_w6_stamps(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_w6_stamp), (size_t)n * 64) == hipSuccess ? 0 : -1;
}
#endif
}  // namespace po
