// Convolutions of the Darknet stack on gfx950 fp32 matrix cores.
//
// po_conv: implicit GEMM  D[m][n] = sum_k A[m][k] * W[n][k]
//   m = output pixel of the launch grid (b,i,j), n = output channel,
//   k = (tap t, input channel c); A[m][(t,c)] = in[b, i*in_step+dh[t], j*in_step+dw[t], c]
//   (zero outside the source).  The same kernel runs the forward conv
//   (taps = the k x k window, BN folded into W/bias, leaky + shortcut in the
//   epilogue) and the input-gradient (dgrad) convs (transposed weights, taps
//   of one stride-parity class).
//
// Tiling: 256 threads = 4 waves, BM x BN block tile, BK input channels per
// k-step, each wave owns (BM/WM) x (BN/WN) built from 32x32 tiles computed
// with v_mfma_f32_32x32x2_f32 (exact fp32, 64 FLOP/clk/SIMD).  Operands go
// global -> registers -> LDS (double buffered, one barrier per k-step).  LDS
// rows are BK floats with their 16-byte chunks XOR-swizzled by row, which
// makes both the ds_write_b128 staging and the ds_read_b128 fragment reads
// bank-conflict free; each lane reads one 16-byte chunk per 4 MFMAs (the k
// order inside a group of 8 is permuted identically for A and B).
#include "conv_common.h"
#include <stdlib.h>
#include <string.h>

namespace {
using po::ConvArgs;

// 16-byte LDS-DMA: lane l's 16 bytes from rsrc+voff land at lds + 16*l
__device__ __forceinline__ void lds_dma16(__amdgpu_buffer_rsrc_t rs, float* lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}

// Split-K reduction + epilogue: one item = 8 output channels of a row.
// The slices are summed in split order (deterministic); an item's loads are
// issued two slices (four 16-byte reads) at a time instead of one dependent
// read per slice.  Every epilogue operand is moved as one 16-byte vector (o
// is a multiple of 4 floats).  32-bit indices: the host checks M * N < 2^31.
// Two forms run the same item code, so their results are bit-identical:
// conv_reduce_k (a kernel of its own, one thread per item) and the in-launch
// reduction of conv_k (the last-arriving slice of a tile, reduce_tile).
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float x, float y, float z, float w) {
  *reinterpret_cast<float4*>(p) = make_float4(x, y, z, w);
}
__device__ __forceinline__ void add4(float4& v, const float4 p) { v.x += p.x; v.y += p.y; v.z += p.z; v.w += p.w; }

// RQ channel quads (8 channels) per item: twice the slice loads in flight.
constexpr int RQ = 2;

struct RedItem {
  uint32_t nib;     // sign bits of the item's y values (bit 4q + c)
  size_t pix;       // destination pixel
  bool live;
};

// Row m, channels n0 .. n0 + 4*RQ - 1 (in_range: m < M and n0 < N): sums the
// ksplit partials in split order and applies the epilogue; max|.| of the
// written values into my / ms / my2.
__device__ __forceinline__ RedItem reduce_item(const ConvArgs& a, int m, int n0, bool in_range, int sh, float& my,
                                               float& ms, float& my2) {
  int b, i, j;
  RedItem r{0u, 0, false};
  r.live = in_range && po::grid_point(a, m, b, i, j);
  if (!r.live) return r;
  r.pix = (size_t)(b * a.Hout + i * a.out_step + a.out_oy) * a.Wout + j * a.out_step + a.out_ox;
  const size_t slice = (size_t)a.M * a.N;
  const float* wp = a.ws + (size_t)m * a.N + n0;
  float4 v[RQ];
#pragma unroll
  for (int q = 0; q < RQ; ++q) v[q] = ld4(wp + 4 * q);
  int s = 1;
  for (; s + 1 < a.ksplit; s += 2) {
    float4 p0[RQ], p1[RQ];
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      p0[q] = ld4(wp + s * slice + 4 * q);
      p1[q] = ld4(wp + (s + 1) * slice + 4 * q);
    }
#pragma unroll
    for (int q = 0; q < RQ; ++q) { add4(v[q], p0[q]); add4(v[q], p1[q]); }
  }
  for (; s < a.ksplit; ++s)
#pragma unroll
    for (int q = 0; q < RQ; ++q) add4(v[q], ld4(wp + s * slice + 4 * q));
  const size_t pix = r.pix;
  const size_t wo = pix * (size_t)(a.Cout_p >> 5) + (n0 >> 5);
  const uint32_t w1 = a.mbits ? a.mbits[wo] : 0u, w2 = a.m2bits ? a.m2bits[wo] : 0u;
#pragma unroll
  for (int q = 0; q < RQ; ++q) {
    const int n = n0 + 4 * q;
    const size_t o = pix * a.Cout_p + n;
    const float rv[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
    const float4 g1 = po::leaky_grad_bits(w1, n);
    const float4 g2 = po::leaky_grad_bits(w2, n);
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 yin = a.accumulate ? ld4(a.y + o) : z4;
    const float4 mk = (!a.mbits && a.mask) ? ld4(a.mask + o) : z4;
    const float4 rs = a.res ? ld4(a.res + o) : z4;
    const float4 mk2 = (a.y2 && !a.m2bits) ? ld4(a.mask2 + o) : z4;
    const float4 bs = a.bias ? ld4(a.bias + n) : z4;
    const float g1v[4] = {g1.x, g1.y, g1.z, g1.w}, g2v[4] = {g2.x, g2.y, g2.z, g2.w};
    const float yiv[4] = {yin.x, yin.y, yin.z, yin.w}, mkv[4] = {mk.x, mk.y, mk.z, mk.w};
    const float rsv[4] = {rs.x, rs.y, rs.z, rs.w}, mk2v[4] = {mk2.x, mk2.y, mk2.z, mk2.w};
    const float bsv[4] = {bs.x, bs.y, bs.z, bs.w};
    float yo[4], so[4], y2o[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float x = __builtin_ldexpf(rv[c], -sh) + bsv[c];
      x = po::leaky_or_id(x, po::act_slope(a.act));
      if (a.accumulate) x += yiv[c];
      const float yv = a.mbits ? x * g1v[c] : (a.mask ? x * po::leaky_grad(mkv[c]) : x);
      yo[c] = yv;
      r.nib |= (yv > 0.f ? 1u : 0u) << (4 * q + c);
      my = fmaxf(my, fabsf(yv));
      so[c] = x + rsv[c];
      if (a.res) ms = fmaxf(ms, fabsf(so[c]));
      y2o[c] = x * (a.m2bits ? g2v[c] : po::leaky_grad(mk2v[c]));
      if (a.y2) my2 = fmaxf(my2, fabsf(y2o[c]));
    }
    if (a.y) st4(a.y + o, yo[0], yo[1], yo[2], yo[3]);
    if (a.res) st4(a.sum + o, so[0], so[1], so[2], so[3]);
    if (a.y2) st4(a.y2 + o, y2o[0], y2o[1], y2o[2], y2o[3]);
  }
  return r;
}

// threads 4k .. 4k+3 hold the 32 channels of one sign-bit word (N % 32 == 0)
__device__ __forceinline__ void reduce_bits(const ConvArgs& a, const RedItem& r, int n0) {
  uint32_t w = r.nib << (4 * RQ * (threadIdx.x & 3));
  w = po::or_group_down<4>(w);
  if (r.live && (threadIdx.x & 3) == 0) a.ybits[r.pix * (a.Cout_p >> 5) + (n0 >> 5)] = w;
}

__global__ __launch_bounds__(256) void conv_reduce_k(const ConvArgs a) {
  const int t0 = (int)blockIdx.x * 256 + (int)threadIdx.x;
  const int n8 = a.N / (4 * RQ);                   // N % 16 == 0 (host check)
  const int tot = a.M * n8;
  const int t = t0 < tot ? t0 : 0;
  const int sh = po::input_shift(a) + (a.prec == 1 ? a.w_shift : 0);
  const int m = t / n8, n0 = (t - m * n8) * 4 * RQ;
  float my = 0.f, ms = 0.f, my2 = 0.f;
  const RedItem r = reduce_item(a, m, n0, t0 < tot, sh, my, ms, my2);
  if (a.ybits) reduce_bits(a, r, n0);
  if (a.y_amax) po::amax_commit(a.y_amax, my);
  if (a.sum_amax) po::amax_commit(a.sum_amax, ms);
  if (a.y2_amax) po::amax_commit(a.y2_amax, my2);
}

// The in-launch reduction of one BM x BN output tile (conv_k, prec 0), run by
// the tile's last-arriving slice: items row-major over the tile, 256 threads
// per pass (BM * BN / 8 is a multiple of 256 for every generic tile, so all
// lanes take every pass and the sign-bit groups stay whole).
template <int BM, int BN>
__device__ __forceinline__ void reduce_tile(const ConvArgs& a, int m0, int n0) {
  constexpr int C8 = BN / (4 * RQ);
  constexpr int ITEMS = BM * C8;
  static_assert(ITEMS % 256 == 0 && C8 % 4 == 0, "reduce_tile: whole passes and sign-bit groups");
  float my = 0.f, ms = 0.f, my2 = 0.f;
#pragma unroll 1
  for (int it = (int)threadIdx.x; it < ITEMS; it += 256) {
    const int r = it / C8, c = it - r * C8;
    const int m = m0 + r, n = n0 + c * 4 * RQ;
    const RedItem ri = reduce_item(a, m, n, m < a.M && n < a.N, 0, my, ms, my2);
    if (a.ybits) reduce_bits(a, ri, n);
  }
  if (a.y_amax) po::amax_commit(a.y_amax, my);
  if (a.sum_amax) po::amax_commit(a.sum_amax, ms);
  if (a.y2_amax) po::amax_commit(a.y2_amax, my2);
}

template <int BM, int BN, int WM, int BK, bool GL>
__global__ __launch_bounds__(256) void conv_k(const ConvArgs a) {
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1, "tile too small for 4 waves of 32x32");
  constexpr int CPR = BK / 4;                  // 16-byte chunks per LDS row
  constexpr int RPP = 256 / CPR;               // rows covered by one load pass of the workgroup
  constexpr int AL = (BM + RPP - 1) / RPP;     // A float4 loads per thread per k-step
  constexpr int BL = (BN + RPP - 1) / RPP;     // B float4 loads per thread per k-step
  constexpr int SW = (BK == 16) ? 2 : 1;       // rows sharing a 256-byte bank line: 1 << SW
  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * BK];
  float* As = smem;                            // [2][BM][BK]
  float* Bs = smem + 2 * BM * BK;              // [2][BN][BK]

  const int wgid = po::xcd_remap();
  const int tn = wgid % a.ntiles_n, tm = wgid / a.ntiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  if (!po::tile_live(a, m0, BM)) return;      // every row of the tile is outside its image's box

  const int tid = threadIdx.x & 255, lane = tid & 63, wave = tid >> 6;   // mask: lets the compiler bound rows
  const int wm = wave / WN, wn = wave % WN;
  const int cth = tid % CPR, rth = tid / CPR;

  // ---- buffer resources over the input tensor and the weights: an offset at or
  // beyond num_records reads zero in hardware, so out-of-image taps and ragged
  // tile rows need neither branches nor clamped addresses
  const uint32_t in_bytes = (uint32_t)__builtin_amdgcn_readfirstlane(a.in_bytes);
  const uint32_t w_bytes = (uint32_t)__builtin_amdgcn_readfirstlane(a.w_bytes);
  const __amdgpu_buffer_rsrc_t in_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.in), 0, in_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t w_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.W), 0, w_bytes, 0x00020000);
  constexpr uint32_t kOOB = 0x80000000u;
  const uint32_t pix_bytes = (uint32_t)a.Cin_p * 4u;

  // ---- A loader state.  Register staging (GL = false): thread (rth, cth)
  // loads chunk cth of rows rth + RPP*r.  LDS-DMA staging (GL = true): the
  // tile is cut into 1 KB pieces (RPI rows); lane L of the wave that owns
  // piece p loads row p*RPI + L/CPR, and the chunk that lands in slot L%CPR
  // of the XOR-swizzled row (the swizzle goes on the source address).
  constexpr int RPI = 64 / CPR;                // rows per 1 KB piece
  constexpr int NPA = BM / RPI, NPB = BN / RPI;
  constexpr int PA = GL ? (NPA + 3) / 4 : AL;  // loader slots per thread / wave
  constexpr int PB = GL ? (NPB + 3) / 4 : BL;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  auto a_row = [&](int r) { return GL ? (wave_u + 4 * r) * RPI + lane / CPR : rth + RPP * r; };
  auto a_chunk = [&](int row) { return GL ? ((lane % CPR) ^ ((row >> SW) & (CPR - 1))) : cth; };
  int a_hi[PA], a_wi[PA];
  uint32_t a_off[PA];
#pragma unroll
  for (int r = 0; r < PA; ++r) {
    const int row = a_row(r);
    const int m = m0 + row;
    int b = 0, i = 0, j = 0;
    const bool ok = (row < BM) && po::grid_point(a, m, b, i, j);
    if (!ok) b = 0;
    a_off[r] = ((uint32_t)b * a.Hin * a.Win) * pix_bytes + a_chunk(row) * 16u;
    // window buffers: shift from output-buffer to input-buffer coordinates
    int sy = 0, sx = 0;
    if (a.out_org) { sy += a.out_org[2 * b]; sx += a.out_org[2 * b + 1]; }
    if (a.in_org) { sy -= a.in_org[2 * b]; sx -= a.in_org[2 * b + 1]; }
    // a row outside the GEMM gets a position no tap can bring into the image
    a_hi[r] = ok ? i * a.in_step + sy : -(1 << 20);
    a_wi[r] = j * a.in_step + sx;
  }
  // ---- B loader state
  const uint32_t wrow_bytes = (uint32_t)a.ntaps * pix_bytes;
  uint32_t b_off[PB];
#pragma unroll
  for (int r = 0; r < PB; ++r) {
    const int row = a_row(r);
    const bool ok = (row < BN) && (n0 + row < a.N);
    b_off[r] = ok ? (uint32_t)(n0 + row) * wrow_bytes + a_chunk(row) * 16u : kOOB;
  }

  float4 ra[GL ? 1 : AL], rb[GL ? 1 : BL];
  auto a_offset = [&](int r, int dh, int dw, uint32_t cb) {
    const int hi = a_hi[r] + dh, wi = a_wi[r] + dw;
    const bool ok = (unsigned)hi < (unsigned)a.Hin && (unsigned)wi < (unsigned)a.Win;
    return ok ? a_off[r] + ((uint32_t)hi * a.Win + wi) * pix_bytes + cb : kOOB;
  };
  auto gload = [&](int tap, int dh, int dw, int c0) {
    const uint32_t cb = (uint32_t)c0 * 4u;
#pragma unroll
    for (int r = 0; r < AL; ++r)
      ra[r] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(in_rs, a_offset(r, dh, dw, cb), 0, 0));
    const uint32_t tb = (uint32_t)tap * pix_bytes + cb;
#pragma unroll
    for (int r = 0; r < BL; ++r)
      rb[r] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(w_rs, b_off[r] + tb, 0, 0));
  };
  auto gload_lds = [&](int buf, int tap, int dh, int dw, int c0) {
    const uint32_t cb = (uint32_t)c0 * 4u;
#pragma unroll
    for (int r = 0; r < PA; ++r) {
      const int p = wave_u + 4 * r;
      if (p < NPA)
        lds_dma16(in_rs, As + (buf * BM + p * RPI) * BK, a_offset(r, dh, dw, cb));
    }
    const uint32_t tb = (uint32_t)tap * pix_bytes + cb;
#pragma unroll
    for (int r = 0; r < PB; ++r) {
      const int p = wave_u + 4 * r;
      if (p < NPB)
        lds_dma16(w_rs, Bs + (buf * BN + p * RPI) * BK, b_off[r] + tb);
    }
  };
  auto swz = [](int row, int chunk) { return (chunk ^ ((row >> SW) & (CPR - 1))) * 4; };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int r = 0; r < AL; ++r) {
      const int row = rth + RPP * r;
      if (row < BM)
        *reinterpret_cast<float4*>(&As[(buf * BM + row) * BK + swz(row, cth)]) = ra[r];
    }
#pragma unroll
    for (int r = 0; r < BL; ++r) {
      const int row = rth + RPP * r;
      if (row < BN)
        *reinterpret_cast<float4*>(&Bs[(buf * BN + row) * BK + swz(row, cth)]) = rb[r];
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int kc = a.Cin_p / BK;
  const int nks_all = a.ntaps * kc;
  // split-K: this workgroup's contiguous range of k-steps
  const int split = blockIdx.y;
  const int ks0 = (int)((int64_t)split * nks_all / a.ksplit);
  const int nks = (int)((int64_t)(split + 1) * nks_all / a.ksplit) - ks0;
  // k-step position: tap (th, tw) and channel offset c0, advanced incrementally
  // k-steps run channel-chunk major, tap minor: the taps of one channel
  // chunk re-read the same (shifted) pixels while they are still in L1/L2
  int tap = ks0 % a.ntaps, c0 = (ks0 / a.ntaps) * BK;
  int th = tap / a.tkw, tw = tap - th * a.tkw;
  if constexpr (GL) {
    gload_lds(0, tap, a.dh0 + th * a.sdh, a.dw0 + tw * a.sdw, c0);
  } else {
    gload(tap, a.dh0 + th * a.sdh, a.dw0 + tw * a.sdw, c0);
    sstore(0);
  }
  __syncthreads();
  const int arow = wm * TM * 32 + (lane & 31);
  const int brow = wn * TN * 32 + (lane & 31);
  const int h = lane >> 5;
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks & 1;
    const bool more = ks + 1 < nks;
    const float* Ab = As + buf * BM * BK;
    const float* Bb = Bs + buf * BN * BK;
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      float4 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = arow + i * 32;
        af[i] = *reinterpret_cast<const float4*>(&Ab[row * BK + swz(row, 2 * g + h)]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = brow + j * 32;
        bf[j] = *reinterpret_cast<const float4*>(&Bb[row * BK + swz(row, 2 * g + h)]);
      }
#ifdef PO_ABLATE_NOLOAD
      if (false) {      // ablation build (tools/): k-steps without staging loads
#else
      if (g == 0 && more) {
#endif
        // issue the next k-step's staging loads behind this group's fragment reads
        if (++tap == a.ntaps) {
          tap = th = tw = 0;
          c0 += BK;
        } else if (++tw == a.tkw) {
          tw = 0;
          ++th;
        }
        if constexpr (GL)
          gload_lds(buf ^ 1, tap, a.dh0 + th * a.sdh, a.dw0 + tw * a.sdw, c0);
        else
          gload(tap, a.dh0 + th * a.sdh, a.dw0 + tw * a.sdw, c0);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i].x, bf[j].x, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i].y, bf[j].y, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i].z, bf[j].z, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i].w, bf[j].w, acc[i][j], 0, 0, 0);
        }
    }
#ifndef PO_ABLATE_NOLOAD
    if constexpr (!GL) {
      if (more) sstore(buf ^ 1);
    }
#endif
    __syncthreads();
  }

  if (a.ksplit > 1) {
    po::store_partials<TM, TN>(a, acc, m0, n0, wm, wn, lane);
    if (!a.tile_ctr) return;                   // the separate reduction kernel follows
    // In-launch reduction (cdna_hip_programming.md, in-launch split-K): every
    // wave drains its partial stores, lane 0 publishes them with an agent-scope
    // release and counts the arrival on the tile's counter; the slice that
    // arrives last acquires and reduces the tile.  Correct for any placement
    // of the slices over XCDs/CUs.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);   // the k-loop buffers are free
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int old = __hip_atomic_fetch_add(a.tile_ctr + wgid, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == a.ksplit - 1;
      if (last) {
        __hip_atomic_store(a.tile_ctr + wgid, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // for the next launch
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      flag[0] = last;
    }
    __syncthreads();
    if (flag[0]) reduce_tile<BM, BN>(a, m0, n0);
    return;
  }
  __shared__ int dst_pix[BM];
  po::conv_epilogue<BM, TM, TN>(a, acc, smem, dst_pix, m0, n0, wm, wn, 0);
}

template <int BM, int BN, int WM, int BK, bool GL>
int launch(const ConvArgs& a, hipStream_t st) {
  ConvArgs b = a;
  b.ntiles_n = po::ceil_div(a.N, BN);
  const int ntiles = po::ceil_div(a.M, BM) * b.ntiles_n;
  // the in-launch split-K reduction needs a counter per output tile
  const bool inl = a.ksplit > 1 && a.tile_ctr && ntiles <= a.tile_ctr_n;
  if (!inl) b.tile_ctr = nullptr;
  hipLaunchKernelGGL((conv_k<BM, BN, WM, BK, GL>), dim3(ntiles, a.ksplit), dim3(256), 0, st, b);
  if (a.ksplit > 1 && !inl) {
    PO_REQUIRE((int64_t)a.M * a.N < (1LL << 31), "po_conv: split-K output too large");
    int rc = po::check_launch("po_conv");
    if (rc) return rc;
    hipLaunchKernelGGL(conv_reduce_k, dim3(po::ceil_div((int64_t)a.M * (a.N / (4 * RQ)), 256)), dim3(256), 0, st, b);
  }
  return po::check_launch("po_conv");
}

template <int BK, bool GL>
int dispatch(const ConvArgs& a, hipStream_t st, int bm, int bn) {
  if (bm == 128 && bn == 128) return launch<128, 128, 2, BK, GL>(a, st);
  if (bm == 64 && bn == 128) return launch<64, 128, 1, BK, GL>(a, st);
  if (bm == 128 && bn == 64) return launch<128, 64, 4, BK, GL>(a, st);
  if (bm == 64 && bn == 64) return launch<64, 64, 2, BK, GL>(a, st);
  if (bm == 128 && bn == 32) return launch<128, 32, 4, BK, GL>(a, st);
  if constexpr (BK == 16 && GL)
    if (bm == 128 && bn == 256) return launch<128, 256, 2, BK, GL>(a, st);
  po::set_error("po_conv: no %dx%d tile", bm, bn);
  return PO_EINVAL;
}

// ADVPATCH_CONV_TILE="BMxBNxBK[g]" forces a tile (tuning experiments only;
// a trailing 'g' selects LDS-DMA staging).
bool forced_tile(int& bm, int& bn, int& bk, int& gl) {
  const char* e = getenv("ADVPATCH_CONV_TILE");
  char g = 0;
  if (!e || sscanf(e, "%dx%dx%d%c", &bm, &bn, &bk, &g) < 3) return false;
  gl = g == 'g';
  return true;
}

// {BM, BN, BK, LDS-DMA staging, precision}.  prec 0 (exact fp32): tiles
// 1..10 stage through registers + ds_write; 11..20 are the same shapes staged
// by LDS-DMA (buffer_load ... lds); 21..28 are the 8-accumulator (64x128 /
// 128x64 per wave) shapes, register- then DMA-staged.  prec 1 (fp16x3,
// conv_h3.hip): 29..45 four-wave kernels with register staging (the A tile is
// split on its way to LDS), 46..52 the LDS-DMA multi-stage kernel (the
// "staging" column = 1; A is split as it is read from LDS), 53..54 the halo
// kernel (staging 2: stride-1 3x3 convs on full maps only), 55..56 the 2-D
// tile halo kernel (staging 3: 3x3 convs of input step 1 or 2 on full maps),
// 57..60 the same with fragment-ordered weights from global (staging 4).
// 61, 62: prec 0 Winograd F(2x2,3x3) (staging 5, conv_wino.hip; BM counts
// 2x2 output tiles): 64 tiles x 32 channels, and 32 tiles x 64 channels with
// LDS-DMA input (62: 4 waves; 63, staging 6: 8 waves, two per SIMD; 64,
// staging 7: 63 with the transform interleaved into the MFMA stream; 65,
// staging 8: 64 with the 16-byte (4-channel) epilogue; 66, staging 11: 65's
// work as 4-wave workgroups in 72 KB of LDS, two per CU; 67, staging 12:
// conv_wino4_k, 64 tiles x 64 channels per 8-wave workgroup with
// register-staged input; 68, staging 13: 67 with the two waves of each SIMD
// staggered by half a k-step); 69, staging 14: conv_halo.hip, a persistent
// 3x3 16 -> 32-channel conv with its max pool fused (8 x 16 output pixels per
// tile, BM = 128); 70, staging 15: conv_wino5_k, tile 68 as a persistent kernel
// pipelined across its units; 71, staging 16: conv_wino6_k, Winograd F(4x4,3x3)
// as a persistent kernel (BM counts 4x4 output tiles); 72, staging 17: tile 71
// on an input transformed beforehand (wino6_pre_k into po_conv_desc.winov); 73, staging 18: conv_wpool.hip,
// tile 69's conv + pool as Winograd F(2x2,3x3) on 16x16x4 MFMAs (BM counts 2x2 tiles).  Retired (see
// retired()): 21..26, 28, 62..64.
constexpr int kTiles[PO_CONV_NTILES][5] = {
    {128, 128, 16, 0, 0}, {128, 128, 32, 0, 0}, {64, 128, 16, 0, 0}, {64, 128, 32, 0, 0}, {128, 64, 16, 0, 0},
    {128, 64, 32, 0, 0},  {64, 64, 16, 0, 0},   {64, 64, 32, 0, 0},  {128, 32, 16, 0, 0}, {128, 32, 32, 0, 0},
    {128, 128, 16, 1, 0}, {128, 128, 32, 1, 0}, {64, 128, 16, 1, 0}, {64, 128, 32, 1, 0}, {128, 64, 16, 1, 0},
    {128, 64, 32, 1, 0},  {64, 64, 16, 1, 0},   {64, 64, 32, 1, 0},  {128, 32, 16, 1, 0}, {128, 32, 32, 1, 0},
    {256, 128, 16, 0, 0}, {256, 128, 32, 0, 0}, {128, 256, 16, 0, 0}, {128, 256, 32, 0, 0},
    {256, 128, 16, 1, 0}, {256, 128, 32, 1, 0}, {128, 256, 16, 1, 0}, {128, 256, 32, 1, 0},
    {128, 128, 16, 0, 1}, {64, 128, 16, 0, 1},  {128, 64, 16, 0, 1},  {64, 64, 16, 0, 1},  {128, 32, 16, 0, 1},
    {128, 128, 32, 0, 1}, {64, 128, 32, 0, 1},  {128, 64, 32, 0, 1},  {64, 64, 32, 0, 1},  {128, 32, 32, 0, 1},
    {256, 128, 32, 0, 1}, {128, 256, 32, 0, 1},
    {128, 128, 64, 0, 1}, {64, 128, 64, 0, 1},  {128, 64, 64, 0, 1},  {64, 64, 64, 0, 1},  {128, 32, 64, 0, 1},
    {128, 128, 32, 1, 1}, {128, 64, 32, 1, 1},  {64, 128, 32, 1, 1},  {64, 64, 32, 1, 1},  {256, 128, 32, 1, 1},
    {128, 128, 16, 1, 1}, {256, 128, 16, 1, 1}, {128, 128, 16, 2, 1}, {128, 64, 16, 2, 1},
    {128, 128, 16, 3, 1}, {128, 64, 16, 3, 1},
    {128, 128, 16, 4, 1}, {128, 64, 16, 4, 1}, {256, 128, 16, 4, 1}, {256, 64, 16, 4, 1},
    {64, 32, 16, 5, 0}, {32, 64, 16, 5, 0}, {32, 64, 16, 6, 0}, {32, 64, 16, 7, 0}, {32, 64, 16, 8, 0},
    {32, 64, 16, 11, 0}, {64, 64, 16, 12, 0}, {64, 64, 16, 13, 0}, {128, 32, 16, 14, 0}, {64, 64, 16, 15, 0},
    {32, 64, 16, 16, 0}, {32, 64, 16, 17, 0}, {32, 32, 16, 18, 0}};
// Tiles no tuned cache or tuner run selected over rounds 1-3 (the 256x128
// shapes, the register-staged and BK-32 128x256 ones, the 32x64 Winograd
// kernels before tile 65); their numbers stay reserved so cached choices keep
// their meaning.
constexpr bool retired(int t) { return (t >= 21 && t <= 26) || t == 28 || (t >= 62 && t <= 64); }
}  // namespace

extern "C" int po_conv_tile_info(int t, int* bm, int* bn, int* bk, int* prec) {
  PO_REQUIRE(t >= 1 && t <= PO_CONV_NTILES && bm && bn && bk, "po_conv_tile_info: bad tile %d", t);
  *bm = kTiles[t - 1][0];
  *bn = kTiles[t - 1][1];
  *bk = kTiles[t - 1][2];
  if (prec) *prec = retired(t) ? -1 : kTiles[t - 1][4];
  return PO_OK;
}

extern "C" int po_conv(const po_conv_desc* d, const float* in, const float* W, const float* bias,
                       float* y_out, const float* res, float* sum_out, const float* mask_y,
                       float* y2_out, const float* mask2, po_stream_t s) {
  PO_REQUIRE(d && in && W, "po_conv: null pointer");
  // y_out may be NULL only when the launch still writes something: the shortcut
  // sum or the sign bits (a forward activation used only as a LeakyReLU mask)
  PO_REQUIRE(y_out || ((sum_out || d->ybits || d->pool_y) && !d->accumulate && !mask_y && !d->mbits && !y2_out),
             "po_conv: y_out may be NULL only for a plain forward conv that writes sum_out, ybits or pool_y");
  PO_REQUIRE(!d->pool_y || (d->pool_argmax && !y_out && !res && !d->accumulate && !mask_y && !d->mbits && !y2_out &&
                            !d->ybits && !d->gbox && !d->in_org && !d->out_org && d->out_step == 1 &&
                            d->out_oy == 0 && d->out_ox == 0 && d->Hg == d->Hout && d->Wg == d->Wout &&
                            d->Hg % 2 == 0 && d->Wg % 2 == 0 && d->ksplit <= 1 && d->N % 4 == 0),
             "po_conv: pool_y needs a plain full-map forward conv (even grid, no split-K, no other outputs)");
  PO_REQUIRE((res == nullptr) == (sum_out == nullptr), "po_conv: res and sum_out must both be set or both NULL");
  PO_REQUIRE((y2_out == nullptr) == (mask2 == nullptr && d->m2bits == nullptr),
             "po_conv: y2_out needs mask2 or m2bits (and neither without y2_out)");
  PO_REQUIRE(!(mask_y && d->mbits) && !(mask2 && d->m2bits), "po_conv: give a mask as floats or as bits, not both");
  PO_REQUIRE(!(d->ybits || d->mbits || d->m2bits) || (d->N % 32 == 0 && d->Cout_p % 32 == 0),
             "po_conv: sign-bit masks need N and Cout_p multiples of 32 (N=%d Cout_p=%d)", d->N, d->Cout_p);
  PO_REQUIRE(d->Cin_p % 16 == 0 && d->Cin_p > 0, "po_conv: Cin_p=%d must be a positive multiple of 16", d->Cin_p);
  PO_REQUIRE(d->N > 0 && d->N % 16 == 0 && d->N <= d->Cout_p, "po_conv: N=%d must be a multiple of 16 <= Cout_p=%d", d->N, d->Cout_p);
  PO_REQUIRE(d->ntaps >= 1 && d->ntaps <= 9, "po_conv: ntaps=%d", d->ntaps);
  PO_REQUIRE(d->B > 0 && d->Hg > 0 && d->Wg > 0 && d->Hin > 0 && d->Win > 0, "po_conv: bad grid");
  PO_REQUIRE((d->Hg - 1) * d->out_step + d->out_oy < d->Hout && (d->Wg - 1) * d->out_step + d->out_ox < d->Wout,
             "po_conv: launch grid writes outside the destination");
  PO_REQUIRE((int64_t)d->B * d->Hout * d->Wout < (1LL << 31), "po_conv: destination too large");
  ConvArgs a;
  a.in = in; a.W = W; a.Wf = d->Wfrag; a.bias = bias; a.y = y_out; a.res = res; a.sum = sum_out; a.mask = mask_y;
  a.y2 = y2_out; a.mask2 = mask2;
  a.in_org = d->in_org; a.out_org = d->out_org; a.gbox = d->gbox;
  PO_REQUIRE(!d->gbox || !d->out_org, "po_conv: gbox needs a full-map destination (out_org NULL)");
  PO_REQUIRE((int64_t)d->B * d->Hout * d->Wout * d->Cout_p < (1LL << 31),
             "po_conv: the destination needs < 2^31 elements (32-bit epilogue offsets)");
  a.prec = d->prec;
  a.w_shift = d->w_shift;
  a.in_amax = d->in_amax;
  a.y_amax = d->y_amax;
  a.sum_amax = d->sum_amax;
  a.y2_amax = d->y2_amax;
  a.ybits = d->ybits;
  a.mbits = d->mbits;
  a.m2bits = d->m2bits;
  PO_REQUIRE(a.prec == 0 || a.prec == 1, "po_conv: prec %d", a.prec);
  PO_REQUIRE(a.prec == 0 || a.in_amax, "po_conv: prec 1 needs the input's max|x| slot (in_amax)");
  PO_REQUIRE(!sum_out || !a.sum_amax || a.sum_amax != a.y_amax, "po_conv: y and sum share an amax slot");
  a.ksplit = d->ksplit > 1 ? d->ksplit : 1;
  a.ws = d->workspace;
  a.tile_ctr = d->tile_ctr;
  a.tile_ctr_n = d->tile_ctr ? d->tile_ctr_n : 0;
  PO_REQUIRE(a.ksplit <= 64 && a.ksplit <= d->ntaps * (d->Cin_p / 16), "po_conv: ksplit %d out of range", a.ksplit);
  PO_REQUIRE(a.ksplit == 1 || a.ws, "po_conv: ksplit > 1 needs a workspace");
  if (d->in_org || d->out_org)
    PO_REQUIRE(d->in_step == 1 && d->out_step == 1 && d->out_oy == 0 && d->out_ox == 0,
               "po_conv: window buffers need in_step = out_step = 1 and no output offset");
  a.B = d->B; a.Hin = d->Hin; a.Win = d->Win; a.Cin_p = d->Cin_p;
  a.Hout = d->Hout; a.Wout = d->Wout; a.Cout_p = d->Cout_p; a.Hg = d->Hg; a.Wg = d->Wg;
  a.in_step = d->in_step; a.out_step = d->out_step; a.out_oy = d->out_oy; a.out_ox = d->out_ox;
  a.ntaps = d->ntaps; a.N = d->N; a.act = d->act; a.accumulate = d->accumulate;
  a.pool_y = d->pool_y;
  a.pool_am = d->pool_argmax;
  a.mrows = d->mrows > 0 ? d->mrows : d->Hg * d->Wg;
  PO_REQUIRE(a.mrows <= d->Hg * d->Wg && (a.mrows == d->Hg * d->Wg || d->gbox),
             "po_conv: mrows %d needs gbox and at most Hg*Wg = %d rows", a.mrows, d->Hg * d->Wg);
  a.M = d->B * a.mrows;
  po::div_magic(a.mrows, a.mg_rows, a.sh_rows);
  po::div_magic(a.Wg, a.mg_wg, a.sh_wg);
  a.ntiles_n = 1;
  const int64_t in_bytes = (int64_t)d->B * d->Hin * d->Win * d->Cin_p * 4;
  // prec 1: w_bytes is one fp16 plane (the lo plane follows it)
  const int64_t w_bytes = (int64_t)d->N * d->ntaps * d->Cin_p * (a.prec == 1 ? 2 : 4);
  PO_REQUIRE(in_bytes < (1LL << 31) && w_bytes < (1LL << 30),
             "po_conv: input (%lld B) must be < 2 GiB and weights (%lld B) < 1 GiB (32-bit buffer offsets)",
             (long long)in_bytes, (long long)w_bytes);
  a.in_bytes = (uint32_t)in_bytes;
  a.w_bytes = (uint32_t)w_bytes;
  // the tap list must be a rectangular grid, row-major, with constant steps
  int tkw = 1;
  while (tkw < d->ntaps && d->dh[tkw] == d->dh[0]) ++tkw;
  PO_REQUIRE(d->ntaps % tkw == 0, "po_conv: taps are not a rectangular grid");
  const int tkh = d->ntaps / tkw;
  a.tkw = tkw;
  a.dh0 = d->dh[0];
  a.dw0 = d->dw[0];
  a.sdh = tkh > 1 ? d->dh[tkw] - d->dh[0] : 0;
  a.sdw = tkw > 1 ? d->dw[1] - d->dw[0] : 0;
  for (int t = 0; t < d->ntaps; ++t)
    PO_REQUIRE(d->dh[t] == a.dh0 + (t / tkw) * a.sdh && d->dw[t] == a.dw0 + (t % tkw) * a.sdw,
               "po_conv: tap %d (%d,%d) breaks the rectangular tap grid", t, d->dh[t], d->dw[t]);
  hipStream_t st = po::stream_of(s);
  int bm, bn, bk, gl = 0;
  PO_REQUIRE(d->tile >= 0 && d->tile <= PO_CONV_NTILES, "po_conv: tile %d out of range", d->tile);
  if (d->tile > 0) {
    PO_REQUIRE(!retired(d->tile), "po_conv: tile %d is retired", d->tile);
    bm = kTiles[d->tile - 1][0];
    bn = kTiles[d->tile - 1][1];
    bk = kTiles[d->tile - 1][2];
    gl = kTiles[d->tile - 1][3];
    PO_REQUIRE(kTiles[d->tile - 1][4] == a.prec, "po_conv: tile %d is not a prec-%d tile", d->tile, a.prec);
    PO_REQUIRE(a.Cin_p % bk == 0, "po_conv: tile %d needs Cin_p %% %d == 0 (Cin_p=%d)", d->tile, bk, a.Cin_p);
  } else if (!forced_tile(bm, bn, bk, gl)) {
    // largest tile that still gives >= 2 workgroups per CU
    const int64_t M = a.M;
    const int N = a.N;
    auto tiles = [&](int tbm, int tbn) { return (int64_t)po::ceil_div(M, tbm) * po::ceil_div(N, tbn); };
    bk = (a.Cin_p % 32 == 0) ? 32 : 16;
    if (N <= 32) { bm = 128; bn = 32; }
    else if (N <= 64) { bn = 64; bm = tiles(128, 64) >= 512 ? 128 : 64; }
    else if (tiles(128, 128) >= 512) { bm = 128; bn = 128; }
    else if (tiles(64, 128) >= 512) { bm = 64; bn = 128; }
    else { bm = 64; bn = 64; }
  }
  while (bk > 16 && a.Cin_p % bk != 0) bk /= 2;
  int rc;
  PO_REQUIRE((a.mrows == a.Hg * a.Wg && !a.pool_y) || gl <= 1 ||
                 ((gl == 5 || (gl >= 11 && gl <= 18)) && a.mrows == a.Hg * a.Wg),
             "po_conv: a compact box grid (mrows) runs on the generic tiles only, a fused pool on those and tiles "
             "61/66/67/68/69/70");
  PO_REQUIRE(!a.pool_y || bm * bn <= 128 * 128,
             "po_conv: a fused pool needs a generic tile of at most 128x128 (got %dx%d)", bm, bn);
  if (a.prec == 1) {
    ConvArgs b = a;
    b.ntiles_n = po::ceil_div(a.N, bn);
    PO_REQUIRE(a.ksplit == 1 || (int64_t)a.M * a.N < (1LL << 31), "po_conv: split-K output too large");
    rc = po::launch_h3(b, st, bm, bn, bk, gl);
    if (rc == PO_OK && a.ksplit > 1) {
      hipLaunchKernelGGL(conv_reduce_k, dim3(po::ceil_div((int64_t)a.M * (a.N / (4 * RQ)), 256)), dim3(256), 0, st, b);
      rc = po::check_launch("po_conv (split-K reduce)");
    }
    return rc;
  }
  if (gl == 14) return po::launch_halo(a, st);
  if (gl == 18) return po::launch_wpool(a, d->Wwino, st);
  if (gl >= 5 && gl <= 8) return po::launch_wino(a, d->Wwino, st, bm, gl >= 6 ? 8 : 4, gl >= 7, gl == 8);
  if (gl >= 11 && gl <= 17 && gl != 14) {
    PO_REQUIRE(gl != 17 || d->winov, "po_conv: tile 72 needs the transformed-input workspace (winov)");
    rc = gl == 16 ? po::launch_wino6(a, d->Wwino6, st)
         : gl == 17 ? po::launch_wino6(a, d->Wwino6, st, d->winov, d->winov_floats)
         : gl == 15 ? po::launch_wino5(a, d->Wwino, st)
         : gl >= 12 ? po::launch_wino4(a, d->Wwino, st, gl == 13)
                    : po::launch_wino(a, d->Wwino, st, bm, 4, false, true, true);
    if (rc == PO_OK && a.ksplit > 1) {
      hipLaunchKernelGGL(conv_reduce_k, dim3(po::ceil_div((int64_t)a.M * (a.N / (4 * RQ)), 256)), dim3(256), 0, st, a);
      rc = po::check_launch("po_conv (winograd split-K reduce)");
    }
    return rc;
  }
  if (bk > 32) bk = 32;
  if (gl) return bk == 32 ? dispatch<32, true>(a, st, bm, bn) : dispatch<16, true>(a, st, bm, bn);
  return bk == 32 ? dispatch<32, false>(a, st, bm, bn) : dispatch<16, false>(a, st, bm, bn);
}
