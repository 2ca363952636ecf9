// po_conv tile 69 (staging 14): a stride-1 3x3 convolution over 16 input
// channels and 32 output channels with its 2x2/2 max pool fused -- the
// first conv after yolov3-tiny's input pool (darknet_v3.py:37-69, layers 2-3
// of yolov3-tiny-15: 208x208, 16 -> 32, maxpool), which the generic tiles
// run as nine one-tap k-steps of 8 MFMAs each with a barrier and a fresh
// 128-row A tile per tap.
//
// Here a persistent workgroup (4 waves) walks 8 x 16-pixel output tiles:
//   * the tile's input patch (10 x 18 pixels x 16 channels, zero outside the
//     image) is loaded ONCE into LDS, the next tile's patch one tile ahead in
//     registers (three 16-byte loads per thread), one barrier per tile;
//   * the weights of the workgroup's 32 output channels live in registers for
//     the whole launch (18 x float4 per lane);
//   * wave w computes output rows 2w, 2w+1 (32 pixels) x 32 channels: 9 taps
//     x 8 v_mfma_f32_32x32x2_f32, the A fragments read from the patch at the
//     tap's offset (2 ds_read_b128 per tap; 20-float pixel stride, so 16
//     consecutive pixels hit 16 distinct 16-byte bank groups);
//   * the 2x2 pool windows lie inside a lane's accumulator rows, so bias,
//     LeakyReLU and conv_pool_epilogue's max rule run in registers and only the
//     pooled value and its argmax byte are stored.
// The MFMA k order (tap-major; step 4g + j pairs channels 8g + j and
// 8g + 4 + j) is conv_k's with BK = 16, and the epilogue arithmetic is
// conv_pool_epilogue's: bit-identical to the generic tiles (test_gpu_halo.py).
#include "conv_common.h"

namespace {
using po::ConvArgs;

constexpr int HR = 8, HC = 16;             // output rows x columns per tile
constexpr int PR = HR + 2, PC = HC + 2;    // input patch rows x columns
constexpr int PS = 20;                     // LDS floats per patch pixel (16 channels + 4 of padding)
constexpr int PATCH = PR * PC * PS;        // floats per patch buffer (14.4 KB)
constexpr int NCH = PR * PC * 4;           // 16-byte chunks per patch (720)
constexpr int LPT = (NCH + 255) / 256;     // chunk loads per thread (3)
constexpr uint32_t kOOB = 0x80000000u;
#ifndef PO_HALO_OCC
#define PO_HALO_OCC 3                      // workgroups per CU (134 VGPRs: 3 waves per SIMD)
#endif

__global__ __launch_bounds__(256, PO_HALO_OCC) void conv_halo_pool_k(const ConvArgs a, int tiles_r, int tiles_c, int ntiles, int xr) {
  __shared__ __attribute__((aligned(16))) float smem[2 * PATCH];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, n = lane & 31;
  const uint32_t in_bytes = (uint32_t)__builtin_amdgcn_readfirstlane(a.in_bytes);
  const __amdgpu_buffer_rsrc_t in_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.in), 0, in_bytes, 0x00020000);

  // weights of output channel n for the lane's half: per tap, channels 4h..4h+3 and 8+4h..8+4h+3
  const float* Wt = reinterpret_cast<const float*>(a.W);
  float4 wq[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int g = 0; g < 2; ++g) wq[t][g] = *reinterpret_cast<const float4*>(Wt + ((size_t)n * 9 + t) * 16 + 8 * g + 4 * h);
  const float bias_n = a.bias ? a.bias[n] : 0.f;
  // tap t -> patch offset (dh + 1, dw + 1), in the launch's tap order
  int toff[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int dh = a.dh0 + (t / 3) * a.sdh, dw = a.dw0 + (t % 3) * a.sdw;
    toff[t] = ((dh + 1) * PC + dw + 1) * PS;
  }
  // the lane's pixel in its wave's two rows
  const int m = lane & 31, yy = m >> 4, xx = m & 15;
  const int abase = ((2 * wave + yy) * PC + xx) * PS + 4 * h;

  float4 ld[LPT];
  auto gload = [&](int tile) {
    const int tc = tile % tiles_c, rest = tile / tiles_c;
    const int tr = rest % tiles_r, b = rest / tiles_r;
    const int y0 = tr * HR - 1, x0 = tc * HC - 1;
#pragma unroll
    for (int r = 0; r < LPT; ++r) {
      const int q = tid + 256 * r;
      const int pp = q >> 2, c = q & 3;
      const int y = y0 + pp / PC, x = x0 + pp % PC;
      const bool ok = q < NCH && (unsigned)y < (unsigned)a.Hin && (unsigned)x < (unsigned)a.Win;
      const uint32_t off = ok ? ((((uint32_t)b * a.Hin + y) * a.Win + x) * 16u + 4u * c) * 4u : kOOB;
      ld[r] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(in_rs, off, 0, 0));
    }
  };
  auto sstore = [&](float* P) {
#pragma unroll
    for (int r = 0; r < LPT; ++r) {
      const int q = tid + 256 * r;
      if (q < NCH) *reinterpret_cast<float4*>(P + (q >> 2) * PS + 4 * (q & 3)) = ld[r];
    }
  };

  float my = 0.f;
  // xr: the workgroups of one XCD walk consecutive tiles at each step (their
  // halos then meet in that XCD's L2); the schedule stays a bijection
  int tile = xr ? po::xcd_remap() : (int)blockIdx.x;
  if (tile < ntiles) gload(tile);
  for (int it = 0; tile < ntiles; ++it) {
    float* P = smem + (it & 1) * PATCH;
    sstore(P);
    __syncthreads();                       // patch complete; the buffer written two tiles ago is free
    const int next = tile + gridDim.x;
    if (next < ntiles) gload(next);        // lands during this tile's MFMAs and epilogue
    floatx16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const float4 a0 = *reinterpret_cast<const float4*>(P + abase + toff[t]);
      const float4 a1 = *reinterpret_cast<const float4*>(P + abase + toff[t] + 8);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, wq[t][0].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, wq[t][0].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.z, wq[t][0].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.w, wq[t][0].w, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.x, wq[t][1].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.y, wq[t][1].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.z, wq[t][1].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.w, wq[t][1].w, acc, 0, 0, 0);
    }
    // epilogue: accumulator row (e & 3) + 8 (e >> 2) + 4h is pixel (yy, xx) of the wave's rows; the pool
    // window of columns x, x+1 (x = 8 grp + 4h + 2q) takes e = 4 grp + 2q (+1) in row 0 and e + 8 (+1) in row 1
    const int tc = tile % tiles_c, rest = tile / tiles_c;
    const int tr = rest % tiles_r, b = rest / tiles_r;
    const int orow = tr * HR + 2 * wave;
    const int Hp = a.Hout >> 1, Wp = a.Wout >> 1;
#pragma unroll
    for (int grp = 0; grp < 2; ++grp)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int e0 = 4 * grp + 2 * q;
        const int ocol = tc * HC + 8 * grp + 4 * h + 2 * q;
        const float v[4] = {acc[e0], acc[e0 + 1], acc[e0 + 8], acc[e0 + 9]};
        float pv = 0.f;
        uint32_t arg = 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float x = v[k] + bias_n;
          x = po::leaky_or_id(x, po::act_slope(a.act));
          if (k == 0 || x > pv || isnan(x)) { pv = x; arg = (uint32_t)k; }
        }
        if (a.act) arg |= 8u | (pv > 0.f ? 0u : 4u);
        if (orow < a.Hout && ocol < a.Wout) {
          const size_t po = (((size_t)b * Hp + (orow >> 1)) * Wp + (ocol >> 1)) * a.Cout_p + n;
          a.pool_y[po] = pv;
          a.pool_am[po] = (int8_t)arg;
          my = fmaxf(my, fabsf(pv));
        }
      }
    tile = next;
  }
  if (a.y_amax) po::amax_commit(a.y_amax, my);
}
}  // namespace

namespace po {
int launch_halo(const ConvArgs& a, hipStream_t st) {
  PO_REQUIRE(a.prec == 0 && a.Cin_p == 16 && a.N == 32 && a.ntaps == 9 && a.tkw == 3 &&
                 (a.sdh == 1 || a.sdh == -1) && (a.sdw == 1 || a.sdw == -1) && a.dh0 == -a.sdh && a.dw0 == -a.sdw,
             "po_conv: tile 69 needs a full 3x3 neighbourhood over Cin_p = 16 into N = 32 channels");
  PO_REQUIRE(a.pool_y && a.pool_am && a.ksplit == 1 && !a.gbox && a.in_step == 1 && a.out_step == 1 &&
                 a.out_oy == 0 && a.out_ox == 0 && !a.in_org && !a.out_org,
             "po_conv: tile 69 runs a fused-pool conv on full maps without split-K");
  PO_REQUIRE(a.Hg == a.Hout && a.Wg == a.Wout && a.Hin == a.Hout && a.Win == a.Wout && a.Hout % 2 == 0 &&
                 a.Wout % 2 == 0 && !a.res && !a.accumulate && !a.mask && !a.mbits && !a.y2 && !a.ybits && !a.y,
             "po_conv: tile 69 needs source, grid and destination of one even size and only the pooled outputs");
  const int tiles_r = ceil_div(a.Hout, HR), tiles_c = ceil_div(a.Wout, HC);
  const int64_t ntiles = (int64_t)a.B * tiles_r * tiles_c;
  PO_REQUIRE(ntiles < (1LL << 31), "po_conv: tile 69: too many tiles");
  // persistent: as many workgroups as the device holds at once (queried once per device)
  const int resident = resident_groups_cached(reinterpret_cast<const void*>(conv_halo_pool_k), 256);
  const int grid = (int)(ntiles < resident ? ntiles : resident);
  static const int xr = [] {
    const char* e = getenv("ADVPATCH_HALO_XCD");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  hipLaunchKernelGGL(conv_halo_pool_k, dim3(grid), dim3(256), 0, st, a, tiles_r, tiles_c, (int)ntiles, xr);
  return check_launch("po_conv (halo pool tile)");
}
}  // namespace po
