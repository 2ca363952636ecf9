// Split-precision ("fp16x3") implicit-GEMM convolution on gfx950 fp16 matrix cores.
//
// Same GEMM as conv_k (conv_igemm.hip): D[m][n] = sum_k A[m][k] * W[n][k] with
// m = output pixel, n = output channel, k = (tap, input channel).  Each fp32
// operand x is represented, after an exact power-of-two scale s that puts the
// tensor's max|x| in [2^13, 2^14), as x*s = hi + lo with
//   hi = fp16_rne(x*s),  lo = fp16_rne(x*s - hi)        (x*s - hi is exact in fp32)
// so x*s is kept to ~22 significant bits (|x*s - hi - lo| <= 2^-22 |x*s|), and
//   A.W ~ Ahi.Whi + Ahi.Wlo + Alo.Whi                   (the dropped Alo.Wlo ~ 2^-22)
// on v_mfma_f32_32x32x16_f16 (fp16 products are exact in fp32; fp32 accumulate).
// Three 32x32x16 MFMAs (3 x 32 cycles) replace eight exact-fp32 32x32x2 MFMAs
// (8 x 64 cycles) per 32x32x16 block: 5.3x the fp32 matrix rate.  The result
// is scaled back by 2^-(shift_in + shift_w) (ldexp, exact) in the epilogue.
//
// Operands: the activations/gradients stay fp32 in HBM; each k-step's A tile
// is loaded through registers, scaled and split into two fp16 LDS images (hi,
// lo).  The weights are split once on the host into fp16 hi/lo planes
// ([2][N][ntaps][Cin_p], pre-scaled by 2^w_shift) and staged as they are.
// The input scale comes from the max|in| slot that the kernels producing the
// input atomicMax'd (po_conv_desc.in_amax).
//
// LDS rows are BK halfs (BK/8 16-byte chunks) with chunks XOR-swizzled by
// (row / rows-per-256B-line), which makes the ds_write_b128 staging and the
// ds_read_b128 fragment reads (lane l: row l&31, chunk 2g + (l>>5)) conflict-free.
#include "conv_common.h"

namespace {
using po::ConvArgs;
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

// Buffer resource (raw, stride 0) over [base, base + bytes): offsets at or past
// `bytes` read zero.
__device__ __forceinline__ i32x4 make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t p = (uint64_t)base;
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)p);
  r[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(p >> 32));
  r[2] = __builtin_amdgcn_readfirstlane((int)bytes);
  r[3] = 0x00020000;
  return r;
}

// 16-byte LDS-DMA (buffer_load_dwordx4 ... lds): lane l's 16 bytes from
// rsrc + voff land at lds + 16 l.  Issued as inline asm so that hipcc's
// wait-count pass, which cannot tell which LDS bytes a DMA writes, does not
// drain every DMA in flight before each ds_read; the kernel orders the DMAs
// itself (counted vmcnt + s_barrier).
__device__ __forceinline__ void lds_dma16(i32x4 rsrc, const void* lds, uint32_t voff) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const char*)lds));
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0), "v"(voff), "s"(rsrc)
               : "memory", "m0");
}

__device__ __forceinline__ uint32_t pk_f16(float a, float b) {
  half2_t h;
  h[0] = (_Float16)a;
  h[1] = (_Float16)b;
  return __builtin_bit_cast(uint32_t, h);
}

// 8 fp32 values times sc (a power of two) -> hi and lo fp16 chunks.  The
// empty asm keeps the compiler from re-deriving fp32(hi) with a second
// conversion of x: it is read back from the packed halves.
__device__ __forceinline__ void split8(const float4 u, const float4 v, float sc, uint4& hi, uint4& lo) {
  float x[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] *= sc;
  uint32_t h[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    h[i] = pk_f16(x[2 * i], x[2 * i + 1]);
    asm volatile("" : "+v"(h[i]));
    const half2_t hh = __builtin_bit_cast(half2_t, h[i]);
    l[i] = pk_f16(x[2 * i] - (float)hh[0], x[2 * i + 1] - (float)hh[1]);
  }
  hi = make_uint4(h[0], h[1], h[2], h[3]);
  lo = make_uint4(l[0], l[1], l[2], l[3]);
}

template <int BM, int BN, int WM, int BK>
__global__ __launch_bounds__(256) void conv_h3_k(const ConvArgs a) {
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1, "tile too small for 4 waves of 32x32");
  static_assert(BK == 16 || BK == 32 || BK == 64, "BK");
  constexpr int CPR = BK / 8;                  // 16-byte chunks (8 halfs) per LDS row
  constexpr int RPP = 256 / CPR;               // rows per staging pass of the workgroup
  constexpr int AL = (BM + RPP - 1) / RPP;     // A passes per k-step
  constexpr int BL = (BN + RPP - 1) / RPP;
  constexpr int SW = (BK == 16) ? 3 : (BK == 32 ? 2 : 1);   // log2(rows per 256-byte bank line)
  // LDS: [2 buffers][hi, lo][BM rows][BK halfs] for A, then the same for B
  constexpr int A_HALFS = BM * BK, B_HALFS = BN * BK;
  __shared__ __attribute__((aligned(16))) _Float16 smem_h[2 * 2 * (A_HALFS + B_HALFS)];
  static_assert(sizeof(smem_h) >= 4 * 4096, "the epilogue needs 16 KB of LDS");
  _Float16* As = smem_h;                       // [2][2][BM][BK]
  _Float16* Bs = smem_h + 4 * A_HALFS;         // [2][2][BN][BK]

  const int wgid = po::xcd_remap();
  const int tn = wgid % a.ntiles_n, tm = wgid / a.ntiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  if (!po::tile_live(a, m0, BM)) return;      // every row of the tile is outside its image's box
  const int tid = threadIdx.x & 255, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int cth = tid % CPR, rth = tid / CPR;
  const int sh_in = po::input_shift(a);
  const float sc_in = __builtin_ldexpf(1.f, sh_in);

  const uint32_t in_bytes = (uint32_t)__builtin_amdgcn_readfirstlane(a.in_bytes);
  const uint32_t w_bytes = (uint32_t)__builtin_amdgcn_readfirstlane(a.w_bytes);
  const __amdgpu_buffer_rsrc_t in_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.in), 0, in_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t w_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.W), 0, 2 * w_bytes, 0x00020000);
  constexpr uint32_t kOOB = 0x80000000u;
  const uint32_t pix_bytes = (uint32_t)a.Cin_p * 4u;     // fp32 input pixel
  const uint32_t wpix_bytes = (uint32_t)a.Cin_p * 2u;    // fp16 weight row per tap

  // ---- A loader: thread (rth, cth) loads channels [8 cth, 8 cth + 8) of rows rth + RPP*r
  int a_hi[AL], a_wi[AL];
  uint32_t a_off[AL];
#pragma unroll
  for (int r = 0; r < AL; ++r) {
    const int row = rth + RPP * r;
    const int m = m0 + row;
    int b = 0, i = 0, j = 0;
    const bool ok = (row < BM) && po::grid_point(a, m, b, i, j);
    if (!ok) b = 0;
    a_off[r] = ((uint32_t)b * a.Hin * a.Win) * pix_bytes + cth * 32u;
    int sy = 0, sx = 0;
    if (a.out_org) { sy += a.out_org[2 * b]; sx += a.out_org[2 * b + 1]; }
    if (a.in_org) { sy -= a.in_org[2 * b]; sx -= a.in_org[2 * b + 1]; }
    a_hi[r] = ok ? i * a.in_step + sy : -(1 << 20);
    a_wi[r] = j * a.in_step + sx;
  }
  // ---- B loader: same thread grid over weight rows; hi plane, lo plane at +w_bytes
  const uint32_t wrow_bytes = (uint32_t)a.ntaps * wpix_bytes;
  uint32_t b_off[BL];
#pragma unroll
  for (int r = 0; r < BL; ++r) {
    const int row = rth + RPP * r;
    const bool ok = (row < BN) && (n0 + row < a.N);
    b_off[r] = ok ? (uint32_t)(n0 + row) * wrow_bytes + cth * 16u : kOOB;
  }

  float4 ra[AL][2];
  uint4 rbh[BL], rbl[BL];
  auto gload = [&](int tap, int dh, int dw, int c0) {
#pragma unroll
    for (int r = 0; r < AL; ++r) {
      const int hi = a_hi[r] + dh, wi = a_wi[r] + dw;
      const bool ok = (unsigned)hi < (unsigned)a.Hin && (unsigned)wi < (unsigned)a.Win;
      const uint32_t o = ok ? a_off[r] + ((uint32_t)hi * a.Win + wi) * pix_bytes + (uint32_t)c0 * 4u : kOOB;
      ra[r][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(in_rs, o, 0, 0));
      ra[r][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(in_rs, o + 16u, 0, 0));
    }
    const uint32_t tb = (uint32_t)tap * wpix_bytes + (uint32_t)c0 * 2u;
#pragma unroll
    for (int r = 0; r < BL; ++r) {
      rbh[r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(w_rs, b_off[r] + tb, 0, 0));
      rbl[r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(w_rs, b_off[r] + tb + w_bytes, 0, 0));
    }
  };
  auto swz = [](int row, int chunk) { return (chunk ^ ((row >> SW) & (CPR - 1))) * 8; };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int r = 0; r < AL; ++r) {
      const int row = rth + RPP * r;
      if (row < BM) {
        uint4 h, l;
        split8(ra[r][0], ra[r][1], sc_in, h, l);
        _Float16* base = As + (buf * 2) * A_HALFS + row * BK + swz(row, cth);
        *reinterpret_cast<uint4*>(base) = h;
        *reinterpret_cast<uint4*>(base + A_HALFS) = l;
      }
    }
#pragma unroll
    for (int r = 0; r < BL; ++r) {
      const int row = rth + RPP * r;
      if (row < BN) {
        _Float16* base = Bs + (buf * 2) * B_HALFS + row * BK + swz(row, cth);
        *reinterpret_cast<uint4*>(base) = rbh[r];
        *reinterpret_cast<uint4*>(base + B_HALFS) = rbl[r];
      }
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
  const int split = blockIdx.y;
  const int ks0 = (int)((int64_t)split * nks_all / a.ksplit);
  const int nks = (int)((int64_t)(split + 1) * nks_all / a.ksplit) - ks0;
  // k-steps run channel-chunk major, tap minor: the taps of one channel
  // chunk re-read the same (shifted) pixels while they are still in L1/L2
  int tap = ks0 % a.ntaps, c0 = (ks0 / a.ntaps) * BK;
  int th = tap / a.tkw, tw = tap - th * a.tkw;
  gload(tap, a.dh0 + th * a.sdh, a.dw0 + tw * a.sdw, c0);
  sstore(0);
  __syncthreads();
  const int arow = wm * TM * 32 + (lane & 31);
  const int brow = wn * TN * 32 + (lane & 31);
  const int h = lane >> 5;
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks & 1;
    const bool more = ks + 1 < nks;
    const _Float16* Ab = As + buf * 2 * A_HALFS;
    const _Float16* Bb = Bs + buf * 2 * B_HALFS;
#pragma unroll
    for (int g = 0; g < BK / 16; ++g) {
      half8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = arow + i * 32;
        const int o = row * BK + swz(row, 2 * g + h);
        ah[i] = *reinterpret_cast<const half8*>(Ab + o);
        al[i] = *reinterpret_cast<const half8*>(Ab + A_HALFS + o);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = brow + j * 32;
        const int o = row * BK + swz(row, 2 * g + h);
        bh[j] = *reinterpret_cast<const half8*>(Bb + o);
        bl[j] = *reinterpret_cast<const half8*>(Bb + B_HALFS + o);
      }
#if defined(PO_ABLATE_NOLOAD) || defined(PO_ABLATE_NOSTORE)
      if (false) {      // ablation builds (tools/): k-steps without staging loads
#else
      if (g == 0 && more) {
#endif
        if (++tap == a.ntaps) {
          tap = th = tw = 0;
          c0 += BK;
        } else if (++tw == a.tkw) {
          tw = 0;
          ++th;
        }
        gload(tap, a.dh0 + th * a.sdh, a.dw0 + tw * a.sdw, c0);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
#ifndef PO_ABLATE_NOSTORE
    if (more) sstore(buf ^ 1);
#endif
    __syncthreads();
  }

  if (a.ksplit > 1) {
    po::store_partials<TM, TN>(a, acc, m0, n0, wm, wn, lane);
    return;
  }
  __shared__ int dst_pix[BM];
  po::conv_epilogue<BM, TM, TN>(a, acc, reinterpret_cast<float*>(smem_h), dst_pix, m0, n0, wm, wn,
                                sh_in + a.w_shift);
}

// LDS-DMA variant: no staging registers.  Each k-step's A tile (fp32) and
// the weights' hi/lo fp16 tiles are copied global -> LDS by buffer_load ... lds
// (16 bytes per lane, 1 KB per wave-instruction, XOR swizzle applied on the
// source address) into an NS-stage ring, NS - 1 k-steps ahead of the MFMAs;
// the A fragments are split into hi/lo as they are read from LDS.  Every wave
// issues the same number D of DMAs per stage (dummy out-of-range copies past
// the last k-step), so "stage ks has landed" is s_waitcnt vmcnt(D * (NS - 2))
// followed by a raw s_barrier (a __syncthreads would drain every stage).
template <int BM, int BN, int WM, int BK, int NS>
__global__ __launch_bounds__(256) void conv_h3d_k(const ConvArgs a) {
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1, "tile too small for 4 waves of 32x32");
  constexpr int RA = BK * 4, RB = BK * 2;          // LDS row bytes: A fp32, B fp16
  constexpr int CPA = RA / 16, CPB = RB / 16;      // 16-byte chunks per row
  constexpr int SWA = RA == 64 ? 2 : (RA == 128 ? 1 : 0);   // log2(rows per 256-byte bank line)
  constexpr int SWB = RB == 32 ? 3 : (RB == 64 ? 2 : 1);
  constexpr int RPA = 1024 / RA, RPB = 1024 / RB;  // rows per 1 KB DMA piece
  constexpr int NPA = BM / RPA, NPB = BN / RPB;    // pieces per tile (per B plane)
  static_assert(NPA % 4 == 0 && NPB % 4 == 0, "every wave must issue the same DMA count");
  constexpr int PA = NPA / 4, PB = NPB / 4;        // pieces per wave
  constexpr int D = PA + 2 * PB;                   // DMAs per wave per stage
  static_assert(D * (NS - 2) <= 63, "vmcnt range");
  constexpr int A_BYTES = BM * RA, B_BYTES = BN * RB;
  constexpr int SB = A_BYTES + 2 * B_BYTES;        // bytes per stage
  static_assert(NS * SB >= 16384, "the epilogue needs 16 KB of LDS");
  // ONE __shared__ array (a second LDS object makes hipcc drain the DMAs
  // before every ds_read): NS stages, then the epilogue's pixel table
  __shared__ __attribute__((aligned(16))) char smem[NS * SB + BM * 4];

  const int wgid = po::xcd_remap();
  const int tn = wgid % a.ntiles_n, tm = wgid / a.ntiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  if (!po::tile_live(a, m0, BM)) return;      // every row of the tile is outside its image's box
  const int tid = threadIdx.x & 255, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int sh_in = po::input_shift(a);
  const float sc_in = __builtin_ldexpf(1.f, sh_in);

  const uint32_t in_bytes = (uint32_t)__builtin_amdgcn_readfirstlane(a.in_bytes);
  const uint32_t w_bytes = (uint32_t)__builtin_amdgcn_readfirstlane(a.w_bytes);
  const i32x4 in_rs = make_rsrc(a.in, in_bytes);
  const i32x4 w_rs = make_rsrc(a.W, 2 * w_bytes);
  constexpr uint32_t kOOB = 0x80000000u;
  const uint32_t pix_bytes = (uint32_t)a.Cin_p * 4u;
  const uint32_t wpix_bytes = (uint32_t)a.Cin_p * 2u;

  // A pieces of this wave: p = wave + 4r, lane -> row p*RPA + lane/CPA and the
  // source chunk that belongs in LDS slot lane%CPA of the swizzled row
  int a_hi[PA], a_wi[PA];
  uint32_t a_off[PA];
#pragma unroll
  for (int r = 0; r < PA; ++r) {
    const int row = (wave + 4 * r) * RPA + lane / CPA;
    const int m = m0 + row;
    int b = 0, i = 0, j = 0;
    const bool ok = po::grid_point(a, m, b, i, j);
    if (!ok) b = 0;
    const int chunk = (lane % CPA) ^ ((row >> SWA) & (CPA - 1));
    a_off[r] = ((uint32_t)b * a.Hin * a.Win) * pix_bytes + chunk * 16u;
    int sy = 0, sx = 0;
    if (a.out_org) { sy += a.out_org[2 * b]; sx += a.out_org[2 * b + 1]; }
    if (a.in_org) { sy -= a.in_org[2 * b]; sx -= a.in_org[2 * b + 1]; }
    a_hi[r] = ok ? i * a.in_step + sy : -(1 << 20);
    a_wi[r] = j * a.in_step + sx;
  }
  const uint32_t wrow_bytes = (uint32_t)a.ntaps * wpix_bytes;
  uint32_t b_off[PB];
#pragma unroll
  for (int r = 0; r < PB; ++r) {
    const int row = (wave + 4 * r) * RPB + lane / CPB;
    const int chunk = (lane % CPB) ^ ((row >> SWB) & (CPB - 1));
    b_off[r] = (n0 + row < a.N) ? (uint32_t)(n0 + row) * wrow_bytes + chunk * 16u : kOOB;
  }
  auto dma = [&](char* lds, i32x4 rs, uint32_t voff) { lds_dma16(rs, lds, voff); };

  const int kc = a.Cin_p / BK;
  const int nks_all = a.ntaps * kc;
  const int split = blockIdx.y;
  const int ks0 = (int)((int64_t)split * nks_all / a.ksplit);
  const int nks = (int)((int64_t)(split + 1) * nks_all / a.ksplit) - ks0;
  // k-steps run channel-chunk major, tap minor: the taps of one channel
  // chunk re-read the same (shifted) pixels while they are still in L1/L2
  int tap = ks0 % a.ntaps, c0 = (ks0 / a.ntaps) * BK;
  int th = tap / a.tkw, tw = tap - th * a.tkw;
  int issued = 0;                               // k-steps issued so far (relative to ks0)
  // issue the DMAs of the next k-step into stage slot issued % NS (out-of-range
  // zero copies once the k-steps are exhausted, to keep the per-wave count)
  auto issue = [&]() {
    const bool live = issued < nks;
    char* st = smem + (issued % NS) * SB;
    const int dh = a.dh0 + th * a.sdh, dw = a.dw0 + tw * a.sdw;
#pragma unroll
    for (int r = 0; r < PA; ++r) {
      const int hi = a_hi[r] + dh, wi = a_wi[r] + dw;
      const bool ok = live && (unsigned)hi < (unsigned)a.Hin && (unsigned)wi < (unsigned)a.Win;
      dma(st + (wave + 4 * r) * 1024, in_rs,
          ok ? a_off[r] + ((uint32_t)hi * a.Win + wi) * pix_bytes + (uint32_t)c0 * 4u : kOOB);
    }
    const uint32_t tb = (uint32_t)tap * wpix_bytes + (uint32_t)c0 * 2u;
#pragma unroll
    for (int r = 0; r < PB; ++r) {
      const uint32_t o = live ? b_off[r] + tb : kOOB;
      dma(st + A_BYTES + (wave + 4 * r) * 1024, w_rs, o);
      dma(st + A_BYTES + B_BYTES + (wave + 4 * r) * 1024, w_rs, o + w_bytes);
    }
    ++issued;
    if (++tap == a.ntaps) {
      tap = th = tw = 0;
      c0 += BK;
    } else if (++tw == a.tkw) {
      tw = 0;
      ++th;
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

#pragma unroll
  for (int s = 0; s < NS - 1; ++s) issue();
  const int arow = wm * TM * 32 + (lane & 31);
  const int brow = wn * TN * 32 + (lane & 31);
  const int h = lane >> 5;
  for (int ks = 0; ks < nks; ++ks) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D * (NS - 2)) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue();                                    // into the slot read during step ks - 1
    const char* st = smem + (ks % NS) * SB;
    const float* Ab = reinterpret_cast<const float*>(st);
    const _Float16* Bh = reinterpret_cast<const _Float16*>(st + A_BYTES);
    const _Float16* Bl = reinterpret_cast<const _Float16*>(st + A_BYTES + B_BYTES);
#pragma unroll
    for (int g = 0; g < BK / 16; ++g) {
      half8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = arow + i * 32;
        const float* rp = Ab + row * BK;
        const int f = (row >> SWA) & (CPA - 1);
        const float4 u = *reinterpret_cast<const float4*>(rp + ((4 * g + 2 * h) ^ f) * 4);
        const float4 v = *reinterpret_cast<const float4*>(rp + ((4 * g + 2 * h + 1) ^ f) * 4);
#ifdef PO_ABLATE_NOSPLIT
        ah[i] = __builtin_bit_cast(half8, u);          // ablation: the LDS bytes as they are
        al[i] = __builtin_bit_cast(half8, v);
#else
        uint4 hi, lo;
        split8(u, v, sc_in, hi, lo);
        ah[i] = __builtin_bit_cast(half8, hi);
        al[i] = __builtin_bit_cast(half8, lo);
#endif
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = brow + j * 32;
        const int o = row * BK + (((2 * g + h) ^ ((row >> SWB) & (CPB - 1))) * 8);
        bh[j] = *reinterpret_cast<const half8*>(Bh + o);
        bl[j] = *reinterpret_cast<const half8*>(Bl + o);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the trailing (dummy) DMAs write LDS
  __syncthreads();

  if (a.ksplit > 1) {
    po::store_partials<TM, TN>(a, acc, m0, n0, wm, wn, lane);
    return;
  }
  po::conv_epilogue<BM, TM, TN>(a, acc, reinterpret_cast<float*>(smem), reinterpret_cast<int*>(smem + NS * SB),
                                m0, n0, wm, wn, sh_in + a.w_shift);
}

template <int BM, int BN, int WM, int BK, int NS>
int launch_dma(const ConvArgs& a, hipStream_t st) {
  ConvArgs b = a;
  b.ntiles_n = po::ceil_div(a.N, BN);
  const int ntiles = po::ceil_div(a.M, BM) * b.ntiles_n;
  hipLaunchKernelGGL((conv_h3d_k<BM, BN, WM, BK, NS>), dim3(ntiles, a.ksplit), dim3(256), 0, st, b);
  return po::check_launch("po_conv (fp16x3, LDS-DMA)");
}

// LDS-DMA tiles: {BM, BN, BK} -> stage count and wave layout
int dispatch_dma(const ConvArgs& a, hipStream_t st, int bm, int bn, int bk) {
  if (bk == 32) {
    if (bm == 128 && bn == 128) return launch_dma<128, 128, 4, 32, 3>(a, st);
    if (bm == 128 && bn == 64) return launch_dma<128, 64, 4, 32, 4>(a, st);
    if (bm == 64 && bn == 128) return launch_dma<64, 128, 2, 32, 4>(a, st);
    if (bm == 64 && bn == 64) return launch_dma<64, 64, 2, 32, 4>(a, st);
    if (bm == 256 && bn == 128) return launch_dma<256, 128, 4, 32, 3>(a, st);
  }
  if (bk == 16) {
    if (bm == 128 && bn == 128) return launch_dma<128, 128, 4, 16, 4>(a, st);
    if (bm == 256 && bn == 128) return launch_dma<256, 128, 4, 16, 4>(a, st);
  }
  po::set_error("po_conv (fp16x3 LDS-DMA): no %dx%dx%d tile", bm, bn, bk);
  return PO_EINVAL;
}

// Halo variant for stride-1 3x3 convolutions on full maps (the forward convs
// and the stride-1 input-gradient convs of the big Darknet stages).  The A
// rows of the nine taps of one channel chunk are the same input pixels
// shifted by dh*W + dw (flat NHWC pixel index), so the chunk's input rows
// [m0 - (W+1), m0 + BM + W + 1) are loaded and split ONCE into an LDS halo
// image, and each tap reads its A fragments from it at a shifted row; a tap
// that leaves the image reads a zero row.  Only the weights are staged per
// k-step (register path, double buffered); the next chunk's halo rows are
// loaded into registers while the current chunk's nine taps run.
template <int BM, int BN, int WM, int WMAX>
__global__ __launch_bounds__(256) void conv_h3h_k(const ConvArgs a) {
  constexpr int BK = 16;
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1, "tile too small for 4 waves of 32x32");
  constexpr int CPR = BK / 8;                  // 16-byte chunks per LDS row
  constexpr int SW = 3;                        // log2(rows per 256-byte bank line) for 32-byte rows
  constexpr int HR = BM + 2 * (WMAX + 1);      // halo rows (largest W)
  constexpr int HZ = HR;                       // the zero row
  constexpr int H_HALFS = (HR + 1) * BK;       // one halo plane
  constexpr int B_HALFS = BN * BK;
  constexpr int HL = (HR * CPR + 255) / 256;   // halo chunk loads per thread
  constexpr int BL = (BN * CPR + 255) / 256;   // weight chunk loads per thread (per plane)
  constexpr int PF = 3;                        // weight k-steps in flight (register ring)
  static_assert(9 % PF == 0, "ring slot of k-step 9c + t must not depend on c");
  __shared__ __attribute__((aligned(16))) _Float16 smem_h[2 * H_HALFS + 4 * B_HALFS];
  static_assert(sizeof(smem_h) >= 4 * 4096, "the epilogue needs 16 KB of LDS");
  _Float16* Hs = smem_h;                       // [hi, lo][HR + 1][BK]
  _Float16* Bs = smem_h + 2 * H_HALFS;         // [2 buffers][hi, lo][BN][BK]

  const int wgid = po::xcd_remap();
  const int tn = wgid % a.ntiles_n, tm = wgid / a.ntiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x & 255, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int W = a.Win, H = a.Hin;
  const int sh_in = po::input_shift(a);
  const float sc_in = __builtin_ldexpf(1.f, sh_in);
  const uint32_t in_bytes = (uint32_t)__builtin_amdgcn_readfirstlane(a.in_bytes);
  const uint32_t w_bytes = (uint32_t)__builtin_amdgcn_readfirstlane(a.w_bytes);
  const __amdgpu_buffer_rsrc_t in_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.in), 0, in_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t w_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.W), 0, 2 * w_bytes, 0x00020000);
  constexpr uint32_t kOOB = 0x80000000u;
  const uint32_t pix_bytes = (uint32_t)a.Cin_p * 4u;
  const uint32_t wpix_bytes = (uint32_t)a.Cin_p * 2u;
  const int hrows = BM + 2 * (W + 1);          // halo rows of this launch
  const int p_lo = m0 - (W + 1);               // flat input pixel of halo row 0

  // halo loader: chunk load q = tid + 256 r -> halo row q / CPR, channel chunk q % CPR
  uint32_t h_off[HL];
#pragma unroll
  for (int r = 0; r < HL; ++r) {
    const int q = tid + 256 * r;
    const int row = q / CPR, p = p_lo + row;
    h_off[r] = (row < hrows && p >= 0 && p < a.M) ? (uint32_t)p * pix_bytes + (q % CPR) * 32u : kOOB;
  }
  const uint32_t wrow_bytes = (uint32_t)a.ntaps * wpix_bytes;
  uint32_t b_off[BL];
#pragma unroll
  for (int r = 0; r < BL; ++r) {
    const int q = tid + 256 * r;
    const int row = q / CPR;
    b_off[r] = (row < BN && n0 + row < a.N) ? (uint32_t)(n0 + row) * wrow_bytes + (q % CPR) * 16u : kOOB;
  }
  float4 rh[HL][2];
  uint4 rbh[PF][BL], rbl[PF][BL];
  auto load_halo = [&](int c0) {
#pragma unroll
    for (int r = 0; r < HL; ++r) {
      const uint32_t o = h_off[r] + (h_off[r] == kOOB ? 0u : (uint32_t)c0 * 4u);
      rh[r][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(in_rs, o, 0, 0));
      rh[r][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(in_rs, o + 16u, 0, 0));
    }
  };
  // weights of k-step (tap, c0) into ring slot `set` (past the end: out of range = zeros, never stored)
  auto load_w = [&](int set, int tap, int c0, bool live) {
    const uint32_t tb = (uint32_t)tap * wpix_bytes + (uint32_t)c0 * 2u;
#pragma unroll
    for (int r = 0; r < BL; ++r) {
      const uint32_t o = live ? b_off[r] + tb : kOOB;
      rbh[set][r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(w_rs, o, 0, 0));
      rbl[set][r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(w_rs, o + w_bytes, 0, 0));
    }
  };
  auto swz = [](int row, int chunk) { return (chunk ^ ((row >> SW) & (CPR - 1))) * 8; };
  auto store_halo = [&]() {
#pragma unroll
    for (int r = 0; r < HL; ++r) {
      const int q = tid + 256 * r;
      const int row = q / CPR;
      if (row < HR) {
        uint4 hh, ll;
        split8(rh[r][0], rh[r][1], sc_in, hh, ll);
        _Float16* base = Hs + row * BK + swz(row, q % CPR);
        *reinterpret_cast<uint4*>(base) = hh;
        *reinterpret_cast<uint4*>(base + H_HALFS) = ll;
      }
    }
  };
  auto store_w = [&](int set, int buf) {
#pragma unroll
    for (int r = 0; r < BL; ++r) {
      const int q = tid + 256 * r;
      const int row = q / CPR;
      if (row < BN) {
        _Float16* base = Bs + (buf * 2) * B_HALFS + row * BK + swz(row, q % CPR);
        *reinterpret_cast<uint4*>(base) = rbh[set][r];
        *reinterpret_cast<uint4*>(base + B_HALFS) = rbl[set][r];
      }
    }
  };

  // per lane, fragment row i and tap t: the swizzled LDS offset of its halo
  // row (the zero row when the tap leaves the image) — no address math in
  // the k-loop
  const int HW = H * W;
  int aoff[TM][9];
  const int h = lane >> 5;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = wm * TM * 32 + i * 32 + (lane & 31);
    const int m = m0 + r;
    const int rem = m % HW;
    const int y = m < a.M ? rem / W : -(1 << 20), x = rem % W;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int dh = a.dh0 + (t / 3) * a.sdh, dw = a.dw0 + (t % 3) * a.sdw;
      const bool ok = (unsigned)(y + dh) < (unsigned)H && (unsigned)(x + dw) < (unsigned)W;
      const int row = ok ? r + W + 1 + dh * W + dw : HZ;
      aoff[i][t] = row * BK + swz(row, h);
    }
  }
  const int brow = wn * TN * 32 + (lane & 31);
  int boff[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) boff[j] = (brow + j * 32) * BK + swz(brow + j * 32, h);

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // k-steps: channel chunk c (16 channels) outside, tap 0..8 inside; this
  // workgroup's split-K range is whole chunks [cb, ce)
  const int nch = a.Cin_p / BK;
  const int cb = (int)((int64_t)blockIdx.y * nch / a.ksplit);
  const int ce = (int)((int64_t)(blockIdx.y + 1) * nch / a.ksplit);
  if (tid < 2 * CPR) *reinterpret_cast<uint4*>(Hs + (tid / CPR) * H_HALFS + HZ * BK + (tid % CPR) * 8) = make_uint4(0, 0, 0, 0);
  load_halo(cb * BK);
#pragma unroll
  for (int s = 0; s < PF; ++s) load_w(s, s, cb * BK, true);         // taps 0..PF-1 of the first chunk
  store_halo();
  store_w(0, 0);
  __syncthreads();
  for (int c = cb; c < ce; ++c) {
    const int c0 = c * BK;
    const bool next_chunk = c + 1 < ce;
    if (next_chunk) load_halo(c0 + BK);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      // k-step g = 9(c - cb) + t of this split's range; B of step g is in ring
      // slot g % PF (= t % PF: 9 % PF == 0), LDS buffer g & 1
      const int cr = (c - cb) & 1;
      const int buf = t & 1 ? cr ^ 1 : cr;               // (9(c - cb) + t) & 1
      const _Float16* Bb = Bs + buf * 2 * B_HALFS;
      half8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        ah[i] = *reinterpret_cast<const half8*>(Hs + aoff[i][t]);
        al[i] = *reinterpret_cast<const half8*>(Hs + H_HALFS + aoff[i][t]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bh[j] = *reinterpret_cast<const half8*>(Bb + boff[j]);
        bl[j] = *reinterpret_cast<const half8*>(Bb + B_HALFS + boff[j]);
      }
      // refill the slot of step g with step g + PF
      const int tp = t + PF;
      const bool more_w = tp < 9 || next_chunk;
      load_w(t % PF, tp < 9 ? tp : tp - 9, tp < 9 ? c0 : c0 + BK, more_w);     // (9c + t) % 3 = t % 3
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
      const bool more = t < 8 || next_chunk;
      if (more) {
        store_w((t + 1) % PF, buf ^ 1);              // step g + 1, loaded PF - 1 steps ago
        if (t == 8) {
          __syncthreads();                         // every wave is done with this chunk's halo
          store_halo();
        }
      }
      __syncthreads();
    }
  }

  if (a.ksplit > 1) {
    po::store_partials<TM, TN>(a, acc, m0, n0, wm, wn, lane);
    return;
  }
  __shared__ int dst_pix[BM];
  po::conv_epilogue<BM, TM, TN>(a, acc, reinterpret_cast<float*>(smem_h), dst_pix, m0, n0, wm, wn,
                                sh_in + a.w_shift);
}

template <int BM, int BN, int WM, int WMAX>
int launch_halo(const ConvArgs& a, hipStream_t st) {
  ConvArgs b = a;
  b.ntiles_n = po::ceil_div(a.N, BN);
  const int ntiles = po::ceil_div(a.M, BM) * b.ntiles_n;
  hipLaunchKernelGGL((conv_h3h_k<BM, BN, WM, WMAX>), dim3(ntiles, a.ksplit), dim3(256), 0, st, b);
  return po::check_launch("po_conv (fp16x3 halo)");
}

int dispatch_halo(const ConvArgs& a, hipStream_t st, int bm, int bn) {
  // eligibility: stride-1 3x3 tap grid on a full map of equal input/output size
  const bool grid3 = a.ntaps == 9 && a.tkw == 3 && (a.sdh == 1 || a.sdh == -1) && (a.sdw == 1 || a.sdw == -1) &&
                     a.dh0 == -a.sdh && a.dw0 == -a.sdw;
  if (!(grid3 && a.in_step == 1 && a.out_step == 1 && a.out_oy == 0 && a.out_ox == 0 && !a.in_org && !a.out_org &&
        !a.gbox &&
        a.Hin == a.Hout && a.Win == a.Wout && a.Hg == a.Hin && a.Wg == a.Win && a.Cin_p % 16 == 0)) {
    po::set_error("po_conv (fp16x3 halo): needs a stride-1 3x3 conv on a full map (no gbox)");
    return PO_EINVAL;
  }
  if (a.Win <= 40) {
    if (bm == 128 && bn == 128) return launch_halo<128, 128, 2, 40>(a, st);
    if (bm == 128 && bn == 64) return launch_halo<128, 64, 4, 40>(a, st);
  } else if (a.Win <= 160) {
    if (bm == 128 && bn == 128) return launch_halo<128, 128, 2, 160>(a, st);
    if (bm == 128 && bn == 64) return launch_halo<128, 64, 4, 160>(a, st);
  } else {
    po::set_error("po_conv (fp16x3 halo): map width %d > 160", a.Win);
    return PO_EINVAL;
  }
  po::set_error("po_conv (fp16x3 halo): no %dx%d tile", bm, bn);
  return PO_EINVAL;
}

// 2-D tile halo variant for 3x3 convs of input step S (1 or 2) on full maps:
// a tile is TH x TW output pixels of one image (BM = TH*TW), so the input halo
// of one channel chunk is (S(TH-1)+3) x (S(TW-1)+3) pixels — 1.41x the tile's
// pixels at S = 1 with 8 x 16 tiles, where the row-contiguous halo of
// conv_h3h_k loads 1 + 2(W+1)/BM rows per tile row (3.4x at W = 152, 5.8x at
// 304) — and strided convs load each input pixel of the tile's footprint once
// instead of once per tap.  The halo is loaded (hardware zero fill outside
// the image) and split into fp16 hi/lo once per chunk, every tap reads its A
// fragments at a precomputed shifted LDS row, the weights run through the
// 3-deep register ring of conv_h3h_k, and the next chunk's halo is fetched
// during the current chunk's nine taps.  No split-K: its partial rows are
// GEMM rows, which 2-D tiles do not enumerate.
template <int BM, int BN, int WM, int TW, int S>
__global__ __launch_bounds__(256) void conv_h3q_k(const ConvArgs a) {
  constexpr int BK = 16;
  constexpr int TH = BM / TW;
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1 && TH * TW == BM, "tile");
  constexpr int CPR = BK / 8;                  // 16-byte chunks per LDS row
  constexpr int SW = 3;                        // log2(rows per 256-byte bank line) for 32-byte rows
  constexpr int HWD = S * (TW - 1) + 3;        // halo width, height, pixels
  constexpr int HHT = S * (TH - 1) + 3;
  constexpr int HP = HWD * HHT;
  constexpr int H_HALFS = HP * BK;             // one halo plane
  constexpr int B_HALFS = BN * BK;
  constexpr int HL = (HP * CPR + 255) / 256;   // halo chunk loads per thread
  constexpr int BL = (BN * CPR + 255) / 256;   // weight chunk loads per thread (per plane)
  constexpr int PF = 3;                        // weight k-steps in flight (register ring)
  static_assert(9 % PF == 0, "ring slot of k-step 9c + t must not depend on c");
  __shared__ __attribute__((aligned(16))) _Float16 smem_h[2 * H_HALFS + 4 * B_HALFS];
  static_assert(sizeof(smem_h) >= 4 * 4096, "the epilogue needs 16 KB of LDS");
  _Float16* Hs = smem_h;                       // [hi, lo][HP][BK]
  _Float16* Bs = smem_h + 2 * H_HALFS;         // [2 buffers][hi, lo][BN][BK]

  const int wgid = po::xcd_remap();
  const int tn = wgid % a.ntiles_n, tm = wgid / a.ntiles_n;
  const int n0 = tn * BN;
  const int tilesx = (a.Wout + TW - 1) / TW, tpi = tilesx * ((a.Hout + TH - 1) / TH);
  const int b = tm / tpi, tr = tm - b * tpi;
  const int oy0 = (tr / tilesx) * TH, ox0 = (tr - (tr / tilesx) * tilesx) * TW;
  const int iy0 = S * oy0 - 1, ix0 = S * ox0 - 1;     // input pixel of halo (0, 0)
  const int tid = threadIdx.x & 255, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int sh_in = po::input_shift(a);
  const float sc_in = __builtin_ldexpf(1.f, sh_in);
  const uint32_t in_bytes = (uint32_t)__builtin_amdgcn_readfirstlane(a.in_bytes);
  const uint32_t w_bytes = (uint32_t)__builtin_amdgcn_readfirstlane(a.w_bytes);
  const __amdgpu_buffer_rsrc_t in_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.in), 0, in_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t w_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.W), 0, 2 * w_bytes, 0x00020000);
  constexpr uint32_t kOOB = 0x80000000u;
  const uint32_t pix_bytes = (uint32_t)a.Cin_p * 4u;
  const uint32_t wpix_bytes = (uint32_t)a.Cin_p * 2u;

  // halo loader: chunk load q = tid + 256 r -> halo pixel q / CPR, channel chunk q % CPR
  uint32_t h_off[HL];
#pragma unroll
  for (int r = 0; r < HL; ++r) {
    const int q = tid + 256 * r;
    const int row = q / CPR;
    const int hy = row / HWD, hx = row - (row / HWD) * HWD;
    const int iy = iy0 + hy, ix = ix0 + hx;
    const bool ok = row < HP && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
    h_off[r] = ok ? ((uint32_t)(b * a.Hin + iy) * a.Win + ix) * pix_bytes + (q % CPR) * 32u : kOOB;
  }
  const uint32_t wrow_bytes = (uint32_t)a.ntaps * wpix_bytes;
  uint32_t b_off[BL];
#pragma unroll
  for (int r = 0; r < BL; ++r) {
    const int q = tid + 256 * r;
    const int row = q / CPR;
    b_off[r] = (row < BN && n0 + row < a.N) ? (uint32_t)(n0 + row) * wrow_bytes + (q % CPR) * 16u : kOOB;
  }
  float4 rh[HL][2];
  uint4 rbh[PF][BL], rbl[PF][BL];
  auto load_halo = [&](int c0) {
#pragma unroll
    for (int r = 0; r < HL; ++r) {
      const uint32_t o = h_off[r] + (h_off[r] == kOOB ? 0u : (uint32_t)c0 * 4u);
      rh[r][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(in_rs, o, 0, 0));
      rh[r][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(in_rs, o + 16u, 0, 0));
    }
  };
  auto load_w = [&](int set, int tap, int c0, bool live) {
    const uint32_t tb = (uint32_t)tap * wpix_bytes + (uint32_t)c0 * 2u;
#pragma unroll
    for (int r = 0; r < BL; ++r) {
      const uint32_t o = live ? b_off[r] + tb : kOOB;
      rbh[set][r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(w_rs, o, 0, 0));
      rbl[set][r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(w_rs, o + w_bytes, 0, 0));
    }
  };
  auto swz = [](int row, int chunk) { return (chunk ^ ((row >> SW) & (CPR - 1))) * 8; };
  auto store_halo = [&]() {
#pragma unroll
    for (int r = 0; r < HL; ++r) {
      const int q = tid + 256 * r;
      const int row = q / CPR;
      if (row < HP) {
        uint4 hh, ll;
        split8(rh[r][0], rh[r][1], sc_in, hh, ll);
        _Float16* base = Hs + row * BK + swz(row, q % CPR);
        *reinterpret_cast<uint4*>(base) = hh;
        *reinterpret_cast<uint4*>(base + H_HALFS) = ll;
      }
    }
  };
  auto store_w = [&](int set, int buf) {
#pragma unroll
    for (int r = 0; r < BL; ++r) {
      const int q = tid + 256 * r;
      const int row = q / CPR;
      if (row < BN) {
        _Float16* base = Bs + (buf * 2) * B_HALFS + row * BK + swz(row, q % CPR);
        *reinterpret_cast<uint4*>(base) = rbh[set][r];
        *reinterpret_cast<uint4*>(base + B_HALFS) = rbl[set][r];
      }
    }
  };

  // per lane, fragment row i (tile pixel (ly, lx)) and tap t: the swizzled
  // LDS offset of its halo pixel (S ly + 1 + dh, S lx + 1 + dw)
  int aoff[TM][9];
  const int h = lane >> 5;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = wm * TM * 32 + i * 32 + (lane & 31);
    const int ly = r / TW, lx = r - (r / TW) * TW;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int dh = a.dh0 + (t / 3) * a.sdh, dw = a.dw0 + (t % 3) * a.sdw;
      const int row = (S * ly + 1 + dh) * HWD + S * lx + 1 + dw;
      aoff[i][t] = row * BK + swz(row, h);
    }
  }
  const int brow = wn * TN * 32 + (lane & 31);
  int boff[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) boff[j] = (brow + j * 32) * BK + swz(brow + j * 32, h);

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nch = a.Cin_p / BK;
  load_halo(0);
#pragma unroll
  for (int s = 0; s < PF; ++s) load_w(s, s, 0, true);                // taps 0..PF-1 of the first chunk
  store_halo();
  store_w(0, 0);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const int c0 = c * BK;
    const bool next_chunk = c + 1 < nch;
    if (next_chunk) load_halo(c0 + BK);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int cr = c & 1;
      const int buf = t & 1 ? cr ^ 1 : cr;               // (9c + t) & 1
      const _Float16* Bb = Bs + buf * 2 * B_HALFS;
      half8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        ah[i] = *reinterpret_cast<const half8*>(Hs + aoff[i][t]);
        al[i] = *reinterpret_cast<const half8*>(Hs + H_HALFS + aoff[i][t]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bh[j] = *reinterpret_cast<const half8*>(Bb + boff[j]);
        bl[j] = *reinterpret_cast<const half8*>(Bb + B_HALFS + boff[j]);
      }
      const int tp = t + PF;
      const bool more_w = tp < 9 || next_chunk;
      load_w(t % PF, tp < 9 ? tp : tp - 9, tp < 9 ? c0 : c0 + BK, more_w);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
      const bool more = t < 8 || next_chunk;
      if (more) {
        store_w((t + 1) % PF, buf ^ 1);
        if (t == 8) {
          __syncthreads();                         // every wave is done with this chunk's halo
          store_halo();
        }
      }
      __syncthreads();
    }
  }

  __shared__ int dst_pix[BM];
  if (tid < BM) {
    const int oy = oy0 + tid / TW, ox = ox0 + tid % TW;
    dst_pix[tid] = (oy < a.Hout && ox < a.Wout) ? (b * a.Hout + oy) * a.Wout + ox : -1;
  }
  po::conv_epilogue<BM, TM, TN>(a, acc, reinterpret_cast<float*>(smem_h), dst_pix, 0, n0, wm, wn,
                                sh_in + a.w_shift, true, false);
}

template <int BM, int BN, int WM, int TW, int S>
int launch_quad(const ConvArgs& a, hipStream_t st) {
  ConvArgs b = a;
  b.ntiles_n = po::ceil_div(a.N, BN);
  constexpr int TH = BM / TW;
  const int64_t ntiles = (int64_t)a.B * po::ceil_div(a.Hout, TH) * po::ceil_div(a.Wout, TW) * b.ntiles_n;
  if (ntiles >= (1LL << 31)) {
    po::set_error("po_conv (fp16x3 2-D halo): too many tiles");
    return PO_EINVAL;
  }
  hipLaunchKernelGGL((conv_h3q_k<BM, BN, WM, TW, S>), dim3((unsigned)ntiles, 1), dim3(256), 0, st, b);
  return po::check_launch("po_conv (fp16x3 2-D halo)");
}

int dispatch_quad(const ConvArgs& a, hipStream_t st, int bm, int bn) {
  // eligibility: a 3x3 tap grid (either orientation) of input step 1 or 2 on
  // full maps, output grid = the whole destination, no split-K, no boxes
  const bool grid3 = a.ntaps == 9 && a.tkw == 3 && (a.sdh == 1 || a.sdh == -1) && (a.sdw == 1 || a.sdw == -1) &&
                     a.dh0 == -a.sdh && a.dw0 == -a.sdw;
  if (!(grid3 && (a.in_step == 1 || a.in_step == 2) && a.out_step == 1 && a.out_oy == 0 && a.out_ox == 0 &&
        !a.in_org && !a.out_org && !a.gbox && a.ksplit == 1 && a.Hg == a.Hout && a.Wg == a.Wout &&
        a.Cin_p % 16 == 0)) {
    po::set_error("po_conv (fp16x3 2-D halo): needs a 3x3 conv of input step 1 or 2 on full maps "
                  "(no gbox, no split-K)");
    return PO_EINVAL;
  }
  if (a.in_step == 1) {
    if (bm == 128 && bn == 128) return launch_quad<128, 128, 2, 16, 1>(a, st);
    if (bm == 128 && bn == 64) return launch_quad<128, 64, 4, 16, 1>(a, st);
  } else {
    if (bm == 128 && bn == 128) return launch_quad<128, 128, 2, 16, 2>(a, st);
    if (bm == 128 && bn == 64) return launch_quad<128, 64, 4, 16, 2>(a, st);
  }
  po::set_error("po_conv (fp16x3 2-D halo): no %dx%d tile", bm, bn);
  return PO_EINVAL;
}

// 2-D tile halo kernel with chunk-staged, fragment-ordered weights (staging
// 4).  The host lays the split weights out in MFMA B-fragment order,
// Wf[plane][N/32][tap][Cin_p/16][64 lanes][8 halves] (lane l: output channel
// 32 nb + (l & 31), input channels 16 c + 8 (l >> 5) .. + 8).  Per channel
// chunk the workgroup loads, at the start of the previous chunk, BOTH the
// chunk's input halo and all nine taps of its weight fragments into
// registers, and writes them to LDS at the chunk boundary (two barriers per
// chunk).  Inside a chunk the nine taps then run from LDS only: no global
// load is waited on and no barrier is crossed between MFMAs, so the loads of
// the next chunk have a whole chunk of MFMA work to land.  B fragment reads
// are one contiguous 1 KB per wave-instruction (conflict-free).
template <int BM, int BN, int WM, int TW, int S>
__global__ __launch_bounds__(256) void conv_h3g_k(const ConvArgs a) {
  constexpr int BK = 16;
  constexpr int TH = BM / TW;
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1 && TH * TW == BM, "tile");
  constexpr int CPR = BK / 8;
  constexpr int SW = 3;
  constexpr int HWD = S * (TW - 1) + 3;
  constexpr int HHT = S * (TH - 1) + 3;
  constexpr int HP = HWD * HHT;
  constexpr int H_HALFS = HP * BK;             // one halo plane
  constexpr int NB = BN / 32;                  // 32-column fragment blocks of the tile
  constexpr int F_HALFS = NB * 9 * 512;        // one weight plane of a chunk (9 taps)
  constexpr int HL = (HP * CPR + 255) / 256;   // halo 16-byte pieces per thread
  constexpr int BQ = (2 * F_HALFS / 8 + 255) / 256;   // weight 16-byte pieces per thread
  static_assert((2 * F_HALFS / 8) % 256 == 0, "weight pieces divide over the workgroup");
  constexpr int SMEM_HALFS = 2 * H_HALFS + 2 * F_HALFS > 8192 ? 2 * H_HALFS + 2 * F_HALFS : 8192;
  __shared__ __attribute__((aligned(16))) _Float16 smem_h[SMEM_HALFS];
  _Float16* Hs = smem_h;                       // [hi, lo][HP][BK]
  _Float16* Fs = smem_h + 2 * H_HALFS;         // [hi, lo][NB][9][64][8]

  const int wgid = po::xcd_remap();
  const int tn = wgid % a.ntiles_n, tm = wgid / a.ntiles_n;
  const int n0 = tn * BN;
  const int tilesx = (a.Wout + TW - 1) / TW, tpi = tilesx * ((a.Hout + TH - 1) / TH);
  const int b = tm / tpi, tr = tm - b * tpi;
  const int oy0 = (tr / tilesx) * TH, ox0 = (tr - (tr / tilesx) * tilesx) * TW;
  const int iy0 = S * oy0 - 1, ix0 = S * ox0 - 1;
  const int tid = threadIdx.x & 255, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int sh_in = po::input_shift(a);
  const float sc_in = __builtin_ldexpf(1.f, sh_in);
  const uint32_t in_bytes = (uint32_t)__builtin_amdgcn_readfirstlane(a.in_bytes);
  const uint32_t w_bytes = (uint32_t)__builtin_amdgcn_readfirstlane(a.w_bytes);
  const __amdgpu_buffer_rsrc_t in_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.in), 0, in_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wf_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.Wf), 0, 2 * w_bytes, 0x00020000);
  constexpr uint32_t kOOB = 0x80000000u;
  const uint32_t pix_bytes = (uint32_t)a.Cin_p * 4u;
  const int nch = a.Cin_p / BK;

  uint32_t h_off[HL];
#pragma unroll
  for (int r = 0; r < HL; ++r) {
    const int q = tid + 256 * r;
    const int row = q / CPR;
    const int hy = row / HWD, hx = row - (row / HWD) * HWD;
    const int iy = iy0 + hy, ix = ix0 + hx;
    const bool ok = row < HP && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
    h_off[r] = ok ? ((uint32_t)(b * a.Hin + iy) * a.Win + ix) * pix_bytes + (q % CPR) * 32u : kOOB;
  }
  // weight piece q = tid + 256 r: plane, block jb, tap t, lane-piece lp (16 bytes)
  uint32_t f_off[BQ];
#pragma unroll
  for (int r = 0; r < BQ; ++r) {
    const int q = tid + 256 * r;
    const int plane = q / (F_HALFS / 8), rem = q - plane * (F_HALFS / 8);
    const int jb = rem / (9 * 64), t = (rem / 64) % 9, lp = rem % 64;
    const int nb = (n0 >> 5) + jb;
    f_off[r] = nb * 32 < a.N ? (uint32_t)plane * w_bytes + (uint32_t)((nb * a.ntaps + t) * nch) * 1024u + lp * 16u
                             : kOOB;
  }
  float4 rh[HL][2];
  uint4 rf[BQ];
  auto load_chunk = [&](int c) {
#pragma unroll
    for (int r = 0; r < BQ; ++r) {
      const uint32_t o = f_off[r] == kOOB ? kOOB : f_off[r] + (uint32_t)c * 1024u;
      rf[r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wf_rs, o, 0, 0));
    }
#pragma unroll
    for (int r = 0; r < HL; ++r) {
      const uint32_t o = h_off[r] + (h_off[r] == kOOB ? 0u : (uint32_t)c * BK * 4u);
      rh[r][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(in_rs, o, 0, 0));
      rh[r][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(in_rs, o + 16u, 0, 0));
    }
  };
  auto swz = [](int row, int chunk) { return (chunk ^ ((row >> SW) & (CPR - 1))) * 8; };
  auto store_chunk = [&]() {
#pragma unroll
    for (int r = 0; r < BQ; ++r) *reinterpret_cast<uint4*>(Fs + (tid + 256 * r) * 8) = rf[r];
#pragma unroll
    for (int r = 0; r < HL; ++r) {
      const int q = tid + 256 * r;
      const int row = q / CPR;
      if (row < HP) {
        uint4 hh, ll;
        split8(rh[r][0], rh[r][1], sc_in, hh, ll);
        _Float16* base = Hs + row * BK + swz(row, q % CPR);
        *reinterpret_cast<uint4*>(base) = hh;
        *reinterpret_cast<uint4*>(base + H_HALFS) = ll;
      }
    }
  };

  int aoff[TM][9];
  const int h = lane >> 5;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = wm * TM * 32 + i * 32 + (lane & 31);
    const int ly = r / TW, lx = r - (r / TW) * TW;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int dh = a.dh0 + (t / 3) * a.sdh, dw = a.dw0 + (t % 3) * a.sdw;
      const int row = (S * ly + 1 + dh) * HWD + S * lx + 1 + dw;
      aoff[i][t] = row * BK + swz(row, h);
    }
  }
  const _Float16* fb = Fs + (wn * TN * 9 * 64 + lane) * 8;    // this lane's fragment of block wn*TN, tap 0

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  load_chunk(0);
  store_chunk();
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const bool next_chunk = c + 1 < nch;
    if (next_chunk) load_chunk(c + 1);          // lands during this chunk's 9 taps
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      half8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        ah[i] = *reinterpret_cast<const half8*>(Hs + aoff[i][t]);
        al[i] = *reinterpret_cast<const half8*>(Hs + H_HALFS + aoff[i][t]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bh[j] = *reinterpret_cast<const half8*>(fb + (j * 9 + t) * 512);
        bl[j] = *reinterpret_cast<const half8*>(fb + F_HALFS + (j * 9 + t) * 512);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
    __syncthreads();                               // every wave is done with this chunk's LDS
    if (next_chunk) {
      store_chunk();
      __syncthreads();
    }
  }

  __shared__ int dst_pix[BM];
  if (tid < BM) {
    const int oy = oy0 + tid / TW, ox = ox0 + tid % TW;
    dst_pix[tid] = (oy < a.Hout && ox < a.Wout) ? (b * a.Hout + oy) * a.Wout + ox : -1;
  }
  po::conv_epilogue<BM, TM, TN>(a, acc, reinterpret_cast<float*>(smem_h), dst_pix, 0, n0, wm, wn,
                                sh_in + a.w_shift, true, false);
}

template <int BM, int BN, int WM, int TW, int S>
int launch_gfrag(const ConvArgs& a, hipStream_t st) {
  ConvArgs b = a;
  b.ntiles_n = po::ceil_div(a.N, BN);
  constexpr int TH = BM / TW;
  const int64_t ntiles = (int64_t)a.B * po::ceil_div(a.Hout, TH) * po::ceil_div(a.Wout, TW) * b.ntiles_n;
  if (ntiles >= (1LL << 31)) {
    po::set_error("po_conv (fp16x3 fragment-weight halo): too many tiles");
    return PO_EINVAL;
  }
  hipLaunchKernelGGL((conv_h3g_k<BM, BN, WM, TW, S>), dim3((unsigned)ntiles, 1), dim3(256), 0, st, b);
  return po::check_launch("po_conv (fp16x3 fragment-weight halo)");
}

int dispatch_gfrag(const ConvArgs& a, hipStream_t st, int bm, int bn) {
  const bool grid3 = a.ntaps == 9 && a.tkw == 3 && (a.sdh == 1 || a.sdh == -1) && (a.sdw == 1 || a.sdw == -1) &&
                     a.dh0 == -a.sdh && a.dw0 == -a.sdw;
  if (!(a.Wf && a.N % 32 == 0 && grid3 && (a.in_step == 1 || a.in_step == 2) && a.out_step == 1 &&
        a.out_oy == 0 && a.out_ox == 0 && !a.in_org && !a.out_org && !a.gbox && a.ksplit == 1 &&
        a.Hg == a.Hout && a.Wg == a.Wout && a.Cin_p % 16 == 0)) {
    po::set_error("po_conv (fp16x3 fragment-weight halo): needs fragment-ordered weights (Wfrag), N %% 32 == 0 "
                  "and a 3x3 conv of input step 1 or 2 on full maps (no gbox, no split-K)");
    return PO_EINVAL;
  }
  if (a.in_step == 1) {
    if (bm == 128 && bn == 128) return launch_gfrag<128, 128, 2, 16, 1>(a, st);
    if (bm == 128 && bn == 64) return launch_gfrag<128, 64, 4, 16, 1>(a, st);
    if (bm == 256 && bn == 128) return launch_gfrag<256, 128, 2, 16, 1>(a, st);
    if (bm == 256 && bn == 64) return launch_gfrag<256, 64, 4, 16, 1>(a, st);
  } else {
    if (bm == 128 && bn == 128) return launch_gfrag<128, 128, 2, 16, 2>(a, st);
    if (bm == 128 && bn == 64) return launch_gfrag<128, 64, 4, 16, 2>(a, st);
  }
  po::set_error("po_conv (fp16x3 fragment-weight halo): no %dx%d tile for input step %d", bm, bn, a.in_step);
  return PO_EINVAL;
}

template <int BM, int BN, int WM, int BK>
int launch(const ConvArgs& a, hipStream_t st) {
  ConvArgs b = a;
  b.ntiles_n = po::ceil_div(a.N, BN);
  const int ntiles = po::ceil_div(a.M, BM) * b.ntiles_n;
  hipLaunchKernelGGL((conv_h3_k<BM, BN, WM, BK>), dim3(ntiles, a.ksplit), dim3(256), 0, st, b);
  return po::check_launch("po_conv (fp16x3)");
}

template <int BK>
int dispatch(const ConvArgs& a, hipStream_t st, int bm, int bn) {
  if (bm == 128 && bn == 128) return launch<128, 128, 2, BK>(a, st);
  if (bm == 64 && bn == 128) return launch<64, 128, 1, BK>(a, st);
  if (bm == 128 && bn == 64) return launch<128, 64, 4, BK>(a, st);
  if (bm == 64 && bn == 64) return launch<64, 64, 2, BK>(a, st);
  if (bm == 128 && bn == 32) return launch<128, 32, 4, BK>(a, st);
  if constexpr (BK <= 32) {
    if (bm == 256 && bn == 128) return launch<256, 128, 2, BK>(a, st);
    if (bm == 128 && bn == 256) return launch<128, 256, 2, BK>(a, st);
  }
  po::set_error("po_conv (fp16x3): no %dx%dx%d tile", bm, bn, BK);
  return PO_EINVAL;
}
}  // namespace

namespace po {
int launch_h3(const ConvArgs& a, hipStream_t st, int bm, int bn, int bk, int staging) {
  if (staging == 4) return dispatch_gfrag(a, st, bm, bn);
  if (staging == 3) return dispatch_quad(a, st, bm, bn);
  if (staging == 2) return dispatch_halo(a, st, bm, bn);
  if (staging == 1) return dispatch_dma(a, st, bm, bn, bk);
  if (bk == 16) return dispatch<16>(a, st, bm, bn);
  if (bk == 32) return dispatch<32>(a, st, bm, bn);
  if (bk == 64) return dispatch<64>(a, st, bm, bn);
  set_error("po_conv (fp16x3): no k-step %d", bk);
  return PO_EINVAL;
}
}  // namespace po
