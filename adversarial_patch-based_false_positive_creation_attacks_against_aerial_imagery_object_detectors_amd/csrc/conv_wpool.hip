// po_conv tile 73 (staging 18): conv_wpool_k, the Winograd F(2x2,3x3) form of
// tile 69 -- a stride-1 3x3 convolution over 16 input channels into 32 output
// channels with its 2x2/2 max pool fused (yolov3-tiny's 208^2 conv 16 -> 32 +
// maxpool, darknet_v3.py:37-69; layers 2-3 of yolov3-tiny-15), bit-identical
// to tile 61 on the same launch.
//
// Tile 69 runs this conv as nine taps x 8 MFMAs per 32 pixels; in F(2x2,3x3) a
// 2x2 output tile -- exactly one pool window -- costs 16 products per channel
// instead of 36.  The generic F(2x2) tiles (61, 65-68) lose that to their
// single k-step (Cin = 16): one input transform, one GEMM pass and a full
// LDS-staged epilogue per workgroup.  Here a persistent workgroup (4 waves,
// two per CU) walks 8 x 16-pixel output tiles (4 x 8 Winograd tiles = 32 pool
// windows) as tile 69 does:
//   * the tile's 10 x 18 x 16 input patch is loaded once (three 16-byte loads
//     per thread, the next tile's one tile ahead in registers) into LDS, its
//     channels stored in the GEMM's k order (below);
//   * thread (Winograd tile, channel pair) forms V = B^T d B (packed pairs,
//     tile 61's operations) into V[xi][tile][16] in LDS;
//   * wave (tile half, channel half) runs the 16 component GEMMs of its 16
//     tiles x 16 output channels on v_mfma_f32_16x16x4_f32, A fragments from V
//     (one ds_read_b128 per component), B fragments (U) held in registers
//     for the whole launch (64 per lane);
//   * the 16x16 accumulator layout puts all 16 components of 4 (tile,
//     channel) pairs in one lane, so Y = A^T M A, bias, LeakyReLU and the pool
//     rule run in registers -- no LDS round trip of M -- and only the pooled
//     value and its argmax byte are stored.
// Bit-identity with tile 61: the fp32 MFMAs are fmaf chains over k (the
// 32x32x2 form in k order per instruction, the 16x16x4 form likewise), and
// lane group g of MFMA step s here meets channel 2s + 8(g&1) + (g>>1), i.e.
// the chain visits channels 0, 8, 1, 9, ..., 7, 15 as tile 61's step s' (lane
// halves h: channels s', 8 + s') does; the transforms, A^T M A, bias, pool
// rule and argmax codes are tile 61's operations in its order
// (tests/test_gpu_wpool.py).
#pragma clang fp contract(off)
#include "conv_common.h"
#include "wino_common.h"

namespace {
using po::ConvArgs;

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int QR = 8, QC = 16;             // output rows x columns per tile
constexpr int QPR = QR + 2, QPC = QC + 2;  // input patch rows x columns
constexpr int QPS = 20;                    // LDS floats per patch pixel (16 channel positions + 4 of padding)
constexpr int QPATCH = QPR * QPC * QPS;    // 3600 floats
constexpr int QNCH = QPR * QPC * 4;        // 16-byte chunks per patch (720)
constexpr int QLPT = (QNCH + 255) / 256;   // chunk loads per thread (3)
constexpr int QT = 32;                     // Winograd tiles (pool windows) per output tile
constexpr int QVS = 20;                    // LDS floats per V row (16 + 4: conflict-free 16-byte reads)
constexpr int QV = 16 * QT * QVS;          // V: 40 KB

// LDS channel position p <-> channel: lane group g = p >> 2 of MFMA step s =
// p & 3 meets channel 2s + 8(g & 1) + (g >> 1)
__device__ __forceinline__ int wp_chan(int p) {
  const int g = p >> 2, s = p & 3;
  return 2 * s + 8 * (g & 1) + (g >> 1);
}

// AMAX: the launch keeps max|pooled value| (ConvArgs.y_amax; fp16x3 consumers only)
template <bool AMAX>
__global__ __launch_bounds__(256, 2) void conv_wpool_k(const ConvArgs a, const float* __restrict__ U, int tiles_r,
                                                       int tiles_c, int ntiles, int xr) {
  __shared__ __attribute__((aligned(16))) float smem[QPATCH + QV];
  float* const P = smem;
  float* const V = smem + QPATCH;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  const int th = wave & 1, cg = wave >> 1;     // the wave's 16 Winograd tiles and 16 output channels
  const int n = 16 * cg + i16;                 // the lane's output channel (GEMM column)
  const uint32_t in_bytes = (uint32_t)__builtin_amdgcn_readfirstlane(a.in_bytes);
  const __amdgpu_buffer_rsrc_t in_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.in), 0, in_bytes, 0x00020000);

  // B fragments for the whole launch: lane (g, n), step s of component xi holds
  // U[xi][wp_chan(4g + s)][n], read from Wwino's fragment order
  // [N/32][Cin_p/16][16][2][64][4] (U[xi][8h + s'][l & 31] at [xi][s' >> 2][32h + (l & 31)][s' & 3])
  float u[16][4];
#pragma unroll
  for (int xi = 0; xi < 16; ++xi)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int c = wp_chan(4 * g + s), h = c >> 3, sp = c & 7;
      u[xi][s] = U[((xi * 2 + (sp >> 2)) * 64 + 32 * h + n) * 4 + (sp & 3)];
    }
  const float bias_n = a.bias ? a.bias[n] : 0.f;
  const int Hp = a.Hout >> 1, Wp = a.Wout >> 1;

  float4 ld[QLPT];
  auto gload = [&](int tile) {
    const int tc = tile % tiles_c, rest = tile / tiles_c;
    const int tr = rest % tiles_r, b = rest / tiles_r;
    const int y0 = tr * QR - 1, x0 = tc * QC - 1;
#pragma unroll
    for (int r = 0; r < QLPT; ++r) {
      const int q = tid + 256 * r;
      const int pp = q >> 2, c = q & 3;
      const int y = y0 + pp / QPC, x = x0 + pp % QPC;
      const bool ok = q < QNCH && (unsigned)y < (unsigned)a.Hin && (unsigned)x < (unsigned)a.Win;
      const uint32_t off = ok ? ((((uint32_t)b * a.Hin + y) * a.Win + x) * 16u + 4u * c) * 4u : kOOB;
      ld[r] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(in_rs, off, 0, 0));
    }
  };
  // chunk c (channels 4c .. 4c+3) -> positions 2c, 2c+1 (channels 4c, 4c+2) and 8+2c, 9+2c (4c+1, 4c+3)
  auto sstore = [&]() {
#pragma unroll
    for (int r = 0; r < QLPT; ++r) {
      const int q = tid + 256 * r;
      if (q < QNCH) {
        float* dst = P + (q >> 2) * QPS + 2 * (q & 3);
        *reinterpret_cast<float2*>(dst) = make_float2(ld[r].x, ld[r].z);
        *reinterpret_cast<float2*>(dst + 8) = make_float2(ld[r].y, ld[r].w);
      }
    }
  };
  // V = B^T d B of Winograd tile t (rows 2tr.., columns 2tc.. of the patch) for
  // channel positions 2pp, 2pp+1: tile 61's operations, in its order
  auto transform = [&]() {
    const int t = tid >> 3, pp = tid & 7;
    const int tr = t >> 3, tc = t & 7;
    f2v d[4][4];
#pragma unroll
    for (int uu = 0; uu < 4; ++uu)
#pragma unroll
      for (int v = 0; v < 4; ++v)
        d[uu][v] = *reinterpret_cast<const f2v*>(P + ((2 * tr + uu) * QPC + 2 * tc + v) * QPS + 2 * pp);
    f2v tt[4][4];
#pragma unroll
    for (int v = 0; v < 4; ++v) {                // columns: B^T over the rows
      tt[0][v] = d[0][v] - d[2][v];
      tt[1][v] = d[1][v] + d[2][v];
      tt[2][v] = d[2][v] - d[1][v];
      tt[3][v] = d[1][v] - d[3][v];
    }
#pragma unroll
    for (int uu = 0; uu < 4; ++uu) {             // rows: B over the columns
      const f2v e[4] = {tt[uu][0] - tt[uu][2], tt[uu][1] + tt[uu][2], tt[uu][2] - tt[uu][1], tt[uu][1] - tt[uu][3]};
#pragma unroll
      for (int v = 0; v < 4; ++v) *reinterpret_cast<f2v*>(V + ((uu * 4 + v) * QT + t) * QVS + 2 * pp) = e[v];
    }
  };

  float my = 0.f;
  const float slope = po::act_slope(a.act);
  const f2v slope2 = {slope, slope}, bias2 = {bias_n, bias_n};
  const bool act = a.act != 0;
  // pooled outputs [B][Hp][Wp][32] floats and argmax bytes (< 2 GiB, host check)
  const uint32_t pool_elems = (uint32_t)(a.B * Hp * Wp) * 32u;
  const __amdgpu_buffer_rsrc_t py_rs = rsrc(a.pool_y, 4u * pool_elems);
  const __amdgpu_buffer_rsrc_t pa_rs = rsrc(a.pool_am, pool_elems);
  int tile = xr ? po::xcd_remap() : (int)blockIdx.x;
  if (tile < ntiles) gload(tile);
  while (tile < ntiles) {
    sstore();                                   // the previous tile's transform read P before its second barrier
    __syncthreads();                            // patch complete; every wave is past the previous tile's GEMM (V free)
    const int next = tile + (int)gridDim.x;
    if (next < ntiles) gload(next);             // lands during this tile's transform, GEMM and epilogue
    transform();
    __syncthreads();                            // V complete
    floatx4 acc[16];
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) {
      acc[xi] = (floatx4){0.f, 0.f, 0.f, 0.f};
      const float4 av = *reinterpret_cast<const float4*>(V + (xi * QT + 16 * th + i16) * QVS + 4 * g);
      acc[xi] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, u[xi][0], acc[xi], 0, 0, 0);
      acc[xi] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, u[xi][1], acc[xi], 0, 0, 0);
      acc[xi] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, u[xi][2], acc[xi], 0, 0, 0);
      acc[xi] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, u[xi][3], acc[xi], 0, 0, 0);
    }
    // epilogue in registers: lane (g, n) holds all components of Winograd tiles
    // 16 th + 4g + e (e = 0..3) for output channel n.  Tiles e = 2ep, 2ep + 1
    // (pool windows px, px + 1 of one row) sit in adjacent accumulator
    // registers, so A^T M A, the bias and the slope product run on the pair
    // (v_pk_add_f32 / v_pk_mul_f32: tile 61's operations per element, in its order)
    const int tc = tile % tiles_c, rest = tile / tiles_c;
    const int tr = rest % tiles_r, b = rest / tiles_r;
    // the lane's pooled pixels: row py, columns px0 + j (j = 2ep + hh), channel n;
    // a dead pixel's offset lies past the buffers (the store is dropped), and
    // the j steps ride in the stores' immediate offsets
    const int py = 4 * tr + 2 * th + (g >> 1), px0 = 8 * tc + 4 * (g & 1);
    const uint32_t base = (((uint32_t)b * Hp + py) * Wp + px0) * 32u + n;
    uint32_t vo[4], vo4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool live = py < Hp && px0 + j < Wp;
      vo[j] = live ? base : kOOB;
      vo4[j] = live ? 4u * base : kOOB;
    }
#pragma unroll
    for (int ep = 0; ep < 2; ++ep) {
      f2v m[16];
#pragma unroll
      for (int xi = 0; xi < 16; ++xi) m[xi] = f2v{acc[xi][2 * ep], acc[xi][2 * ep + 1]};
      f2v s0[4], s1[4];                         // A^T m A, A^T = [[1,1,1,0],[0,1,-1,-1]] (tile 61)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        s0[v] = m[0 * 4 + v] + m[1 * 4 + v] + m[2 * 4 + v];
        s1[v] = m[1 * 4 + v] - m[2 * 4 + v] - m[3 * 4 + v];
      }
      f2v x[4] = {s0[0] + s0[1] + s0[2], s0[1] - s0[2] - s0[3], s1[0] + s1[1] + s1[2], s1[1] - s1[2] - s1[3]};
      f2v xs[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        x[k] = x[k] + bias2;
        xs[k] = x[k] * slope2;                  // leaky_or_id(x) = maximum(x, x * slope)
      }
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int j = 2 * ep + hh;
        float pv = 0.f;
        uint32_t arg = 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float xv = __builtin_elementwise_maximum(x[k][hh], xs[k][hh]);
          if (k == 0 || xv > pv || isnan(xv)) { pv = xv; arg = (uint32_t)k; }
        }
        if (act) arg |= 8u | (pv > 0.f ? 0u : 4u);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, pv), py_rs, vo4[j], 128 * j, 0);
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)arg, pa_rs, vo[j], 32 * j, 0);
        if constexpr (AMAX) my = fmaxf(my, vo[j] != kOOB ? fabsf(pv) : 0.f);
      }
    }
    tile = next;
  }
  if constexpr (AMAX) po::amax_commit(a.y_amax, my);
}
}  // namespace

namespace po {
int launch_wpool(const ConvArgs& a, const float* U, hipStream_t st) {
  PO_REQUIRE(U, "po_conv: tile 73 needs the F(2x2,3x3) weights (Wwino)");
  PO_REQUIRE(a.prec == 0 && a.Cin_p == 16 && a.N == 32 && a.Cout_p == 32 && a.ntaps == 9 && a.tkw == 3 &&
                 (a.sdh == 1 || a.sdh == -1) && (a.sdw == 1 || a.sdw == -1) && a.dh0 == -a.sdh && a.dw0 == -a.sdw,
             "po_conv: tile 73 needs a full 3x3 neighbourhood over Cin_p = 16 into N = Cout_p = 32 channels");
  PO_REQUIRE(a.pool_y && a.pool_am && a.ksplit == 1 && !a.gbox && a.in_step == 1 && a.out_step == 1 &&
                 a.out_oy == 0 && a.out_ox == 0 && !a.in_org && !a.out_org,
             "po_conv: tile 73 runs a fused-pool conv on full maps without split-K");
  PO_REQUIRE(a.Hg == a.Hout && a.Wg == a.Wout && a.Hin == a.Hout && a.Win == a.Wout && a.Hout % 2 == 0 &&
                 a.Wout % 2 == 0 && !a.res && !a.accumulate && !a.mask && !a.mbits && !a.y2 && !a.ybits && !a.y,
             "po_conv: tile 73 needs source, grid and destination of one even size and only the pooled outputs");
  const int tiles_r = ceil_div(a.Hout, QR), tiles_c = ceil_div(a.Wout, QC);
  const int64_t ntiles = (int64_t)a.B * tiles_r * tiles_c;
  PO_REQUIRE(ntiles < (1LL << 31), "po_conv: tile 73: too many tiles");
  PO_REQUIRE((int64_t)a.B * (a.Hout / 2) * (a.Wout / 2) * 32 * 4 < (1LL << 31),
             "po_conv: tile 73: pooled output must be < 2 GiB");
  const bool amax = a.y_amax != nullptr;
  const void* fn = amax ? reinterpret_cast<const void*>(conv_wpool_k<true>) : reinterpret_cast<const void*>(conv_wpool_k<false>);
  const int resident = resident_groups_cached(fn, 256);
  const int grid = (int)(ntiles < resident ? ntiles : resident);
  static const int xr = [] {
    const char* e = getenv("ADVPATCH_HALO_XCD");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  if (amax)
    hipLaunchKernelGGL(conv_wpool_k<true>, dim3(grid), dim3(256), 0, st, a, U, tiles_r, tiles_c, (int)ntiles, xr);
  else
    hipLaunchKernelGGL(conv_wpool_k<false>, dim3(grid), dim3(256), 0, st, a, U, tiles_r, tiles_c, (int)ntiles, xr);
  return check_launch("po_conv (Winograd pool tile)");
}
}  // namespace po
