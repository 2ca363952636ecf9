// Convolutions of the Darknet stack on gfx950 fp32 matrix cores.
//
// po_conv: implicit GEMM  D[m][n] = sum_k A[m][k] * W[n][k]
//   m = output pixel of the launch grid (b,i,j), n = output channel,
//   k = (tap t, input channel c); A[m][(t,c)] = in[b, i*in_step+dh[t], j*in_step+dw[t], c]
//   (zero outside the source).  The same kernel runs the forward conv
//   (taps = the k x k window, BN folded into W/bias, leaky + shortcut in the
//   epilogue) and the input-gradient (dgrad) convs (flipped/transposed weights;
//   stride-2 dgrad is split into 4 parity classes with 1/2/2/4 taps each).
//
// Tiling: 256 threads = 4 waves, BM x BN block tile, BK = 16 channels per
// k-step, each wave owns (BM/WM) x (BN/WN) made of 32x32 tiles computed with
// v_mfma_f32_32x32x2_f32 (exact fp32, 64 FLOP/clk/SIMD).  Operands are staged
// global -> registers -> LDS (double buffered, one barrier per k-step); each
// lane reads its A/B fragments as one ds_read_b128 per 4 MFMAs (the k order
// inside a group of 8 is permuted identically for A and B).
#include "common.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {
constexpr int BK = 16;
constexpr int LDK = 20;  // padded LDS row (floats): conflict-free ds_read_b128 / ds_write_b128

struct ConvArgs {
  const float* in;
  const float* W;
  const float* bias;
  float* y;
  const float* res;
  float* sum;
  const float* mask;
  int B, Hin, Win, Cin_p, Hout, Wout, Cout_p, Hg, Wg;
  int in_step, out_step, out_oy, out_ox;
  int ntaps, N, act, accumulate;
  int M, ntiles_n, kc;  // kc = Cin_p / BK
  int dh[9], dw[9];
};

template <int BM, int BN, int WM>
__global__ __launch_bounds__(256) void conv_k(const ConvArgs a) {
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1, "tile too small for 4 waves of 32x32");
  constexpr int AL = BM / 64;                  // float4 A loads per thread per k-step
  constexpr int BLN = BN * 4;                  // float4 B loads per k-step
  constexpr int BL = (BLN + 255) / 256;
  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * LDK];
  float* As = smem;                            // [2][BM][LDK]
  float* Bs = smem + 2 * BM * LDK;             // [2][BN][LDK]

  // XCD-aware bijective remap: consecutive logical tiles share an XCD's L2
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + orig / 8;
  const int tn = wgid % a.ntiles_n, tm = wgid / a.ntiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int HgWg = a.Hg * a.Wg;

  // ---- A loader state: rows (tid>>2) + 64*r, float4 column (tid&3)
  const int c4 = tid & 3;
  int a_hi[AL], a_wi[AL];
  size_t a_img[AL];
  bool a_ok[AL];
#pragma unroll
  for (int r = 0; r < AL; ++r) {
    const int m = m0 + (tid >> 2) + 64 * r;
    a_ok[r] = m < a.M;
    const int mm = a_ok[r] ? m : 0;
    const int b = mm / HgWg, rem = mm - b * HgWg;
    const int i = rem / a.Wg, j = rem - i * a.Wg;
    a_img[r] = (size_t)b * a.Hin * a.Win;
    a_hi[r] = i * a.in_step;
    a_wi[r] = j * a.in_step;
  }
  // ---- B loader state
  const size_t wrow = (size_t)a.ntaps * a.Cin_p;
  int b_row[BL];
  bool b_ok[BL];
#pragma unroll
  for (int r = 0; r < BL; ++r) {
    const int f = tid + 256 * r;
    b_row[r] = f >> 2;
    b_ok[r] = (f < BLN) && (n0 + b_row[r] < a.N);
  }

  float4 ra[AL], rb[BL];
  auto gload = [&](int tap, int c0) {
    const int dh = a.dh[tap], dw = a.dw[tap];
#pragma unroll
    for (int r = 0; r < AL; ++r) {
      const int hi = a_hi[r] + dh, wi = a_wi[r] + dw;
      if (a_ok[r] && hi >= 0 && hi < a.Hin && wi >= 0 && wi < a.Win) {
        const float* p = a.in + (a_img[r] + (size_t)hi * a.Win + wi) * a.Cin_p + c0 + c4 * 4;
        ra[r] = *reinterpret_cast<const float4*>(p);
      } else {
        ra[r] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int r = 0; r < BL; ++r) {
      if (b_ok[r]) {
        const float* p = a.W + (size_t)(n0 + b_row[r]) * wrow + (size_t)tap * a.Cin_p + c0 + c4 * 4;
        rb[r] = *reinterpret_cast<const float4*>(p);
      } else {
        rb[r] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int r = 0; r < AL; ++r)
      *reinterpret_cast<float4*>(&As[(buf * BM + (tid >> 2) + 64 * r) * LDK + c4 * 4]) = ra[r];
#pragma unroll
    for (int r = 0; r < BL; ++r)
      if (tid + 256 * r < BLN)
        *reinterpret_cast<float4*>(&Bs[(buf * BN + b_row[r]) * LDK + c4 * 4]) = rb[r];
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nks = a.ntaps * a.kc;
  int tap = 0, c0 = 0;
  gload(0, 0);
  sstore(0);
  __syncthreads();
  const int arow = wm * TM * 32 + (lane & 31);
  const int brow = wn * TN * 32 + (lane & 31);
  const int koff = 4 * (lane >> 5);
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks & 1;
    const bool more = ks + 1 < nks;
    if (more) {
      c0 += BK;
      if (c0 == a.Cin_p) { c0 = 0; ++tap; }
      gload(tap, c0);
    }
    const float* Ab = As + buf * BM * LDK;
    const float* Bb = Bs + buf * BN * LDK;
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      float4 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const float4*>(&Ab[(arow + i * 32) * LDK + g * 8 + koff]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bf[j] = *reinterpret_cast<const float4*>(&Bb[(brow + j * 32) * LDK + g * 8 + koff]);
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
    if (more) sstore(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: destination pixel offsets of the BM tile rows via LDS
  int* dst_pix = reinterpret_cast<int*>(smem);
  if (tid < BM) {
    const int m = m0 + tid;
    int o = -1;
    if (m < a.M) {
      const int b = m / HgWg, rem = m - b * HgWg;
      const int i = rem / a.Wg, j = rem - i * a.Wg;
      o = (b * a.Hout + i * a.out_step + a.out_oy) * a.Wout + j * a.out_step + a.out_ox;
    }
    dst_pix[tid] = o;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * TN * 32 + j * 32 + (lane & 31);
      if (n >= a.N) continue;
      const float bv = a.bias ? a.bias[n] : 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = wm * TM * 32 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        const int pix = dst_pix[row];
        if (pix < 0) continue;
        const size_t o = (size_t)pix * a.Cout_p + n;
        float v = acc[i][j][e] + bv;
        if (a.act) v = po::leaky(v);
        if (a.accumulate) v += a.y[o];
        if (a.mask) v *= po::leaky_grad(a.mask[o]);
        a.y[o] = v;
        if (a.res) a.sum[o] = v + a.res[o];
      }
    }
}

template <int BM, int BN, int WM>
int launch(const ConvArgs& a, hipStream_t st) {
  ConvArgs b = a;
  b.ntiles_n = po::ceil_div(a.N, BN);
  const int ntiles = po::ceil_div(a.M, BM) * b.ntiles_n;
  hipLaunchKernelGGL((conv_k<BM, BN, WM>), dim3(ntiles), dim3(256), 0, st, b);
  return po::check_launch("po_conv");
}

// ------------------------------------------------------------------------
// First layer: 3 input channels (NCHW image), 3x3, VALU direct convolution.
// ------------------------------------------------------------------------
template <int CO>
__global__ __launch_bounds__(256) void first_fwd_k(const float* __restrict__ img, int B, int H, int W,
                                                   int stride, int Ho, int Wo,
                                                   const float* __restrict__ Wt,
                                                   const float* __restrict__ bias, int Cout,
                                                   int Cout_p, int act, float* __restrict__ y) {
  __shared__ float ws[CO * 27];
  __shared__ float bs[CO];
  for (int t = threadIdx.x; t < CO * 27; t += 256) ws[t] = (t / 27) < Cout ? Wt[t] : 0.f;
  for (int t = threadIdx.x; t < CO; t += 256) bs[t] = (t < Cout && bias) ? bias[t] : 0.f;
  __syncthreads();
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= (int64_t)B * Ho * Wo) return;
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
  float* yp = y + (size_t)p * Cout_p;
#pragma unroll
  for (int co4 = 0; co4 < CO; co4 += 4) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 27; ++k) s += ws[(co4 + u) * 27 + k] * x[k];
      s += bs[co4 + u];
      v[u] = act ? po::leaky(s) : s;
    }
    *reinterpret_cast<float4*>(yp + co4) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

template <int CO>
__global__ __launch_bounds__(256) void first_dgrad_k(const float* __restrict__ D, int B, int H, int W,
                                                     int stride, int Ho, int Wo,
                                                     const float* __restrict__ Wt, int Cout,
                                                     int Cout_p, float* __restrict__ dimg) {
  __shared__ float ws[CO * 27];
  for (int t = threadIdx.x; t < CO * 27; t += 256) ws[t] = (t / 27) < Cout ? Wt[t] : 0.f;
  __syncthreads();
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= (int64_t)B * H * W) return;
  const int b = (int)(p / ((int64_t)H * W));
  const int rem = (int)(p - (int64_t)b * H * W);
  const int h = rem / W, w = rem % W;
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
      const float* dp = D + (((size_t)b * Ho + ho) * Wo + wo) * Cout_p;
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
  float* o = dimg + (size_t)b * 3 * plane + (size_t)h * W + w;
  o[0] = d0;
  o[plane] = d1;
  o[2 * plane] = d2;
}
}  // namespace

extern "C" int po_conv(const po_conv_desc* d, const float* in, const float* W, const float* bias,
                       float* y_out, const float* res, float* sum_out, const float* mask_y,
                       po_stream_t s) {
  PO_REQUIRE(d && in && W && y_out, "po_conv: null pointer");
  PO_REQUIRE((res == nullptr) == (sum_out == nullptr), "po_conv: res and sum_out must both be set or both NULL");
  PO_REQUIRE(d->Cin_p % BK == 0 && d->Cin_p > 0, "po_conv: Cin_p=%d must be a positive multiple of %d", d->Cin_p, BK);
  PO_REQUIRE(d->N > 0 && d->N % 16 == 0 && d->N <= d->Cout_p, "po_conv: N=%d must be a multiple of 16 <= Cout_p=%d", d->N, d->Cout_p);
  PO_REQUIRE(d->ntaps >= 1 && d->ntaps <= 9, "po_conv: ntaps=%d", d->ntaps);
  PO_REQUIRE(d->B > 0 && d->Hg > 0 && d->Wg > 0 && d->Hin > 0 && d->Win > 0, "po_conv: bad grid");
  PO_REQUIRE((d->Hg - 1) * d->out_step + d->out_oy < d->Hout && (d->Wg - 1) * d->out_step + d->out_ox < d->Wout,
             "po_conv: launch grid writes outside the destination");
  PO_REQUIRE((int64_t)d->B * d->Hout * d->Wout < (1LL << 31), "po_conv: destination too large");
  ConvArgs a;
  a.in = in; a.W = W; a.bias = bias; a.y = y_out; a.res = res; a.sum = sum_out; a.mask = mask_y;
  a.B = d->B; a.Hin = d->Hin; a.Win = d->Win; a.Cin_p = d->Cin_p;
  a.Hout = d->Hout; a.Wout = d->Wout; a.Cout_p = d->Cout_p; a.Hg = d->Hg; a.Wg = d->Wg;
  a.in_step = d->in_step; a.out_step = d->out_step; a.out_oy = d->out_oy; a.out_ox = d->out_ox;
  a.ntaps = d->ntaps; a.N = d->N; a.act = d->act; a.accumulate = d->accumulate;
  a.M = d->B * d->Hg * d->Wg;
  a.kc = d->Cin_p / BK;
  a.ntiles_n = 1;
  for (int t = 0; t < 9; ++t) {
    a.dh[t] = t < d->ntaps ? d->dh[t] : 0;
    a.dw[t] = t < d->ntaps ? d->dw[t] : 0;
  }
  hipStream_t st = po::stream_of(s);
  // tile choice: largest tile that still gives >= 2 workgroups per CU
  const int64_t M = a.M;
  const int N = a.N;
  auto tiles = [&](int bm, int bn) { return (int64_t)po::ceil_div(M, bm) * po::ceil_div(N, bn); };
  if (N <= 32) {
    return launch<128, 32, 4>(a, st);
  }
  if (N <= 64) {
    if (tiles(128, 64) >= 512) return launch<128, 64, 4>(a, st);
    return launch<64, 64, 2>(a, st);
  }
  if (tiles(128, 128) >= 512) return launch<128, 128, 2>(a, st);
  if (tiles(64, 128) >= 512) return launch<64, 128, 1>(a, st);
  return launch<64, 64, 2>(a, st);
}

extern "C" int po_conv_first_fwd(const float* img, int B, int H, int W, int stride, const float* Wt,
                                 const float* bias, int Cout, int Cout_p, int act, float* y,
                                 po_stream_t s) {
  PO_REQUIRE(img && Wt && y, "po_conv_first_fwd: null pointer");
  PO_REQUIRE(stride == 1 || stride == 2, "po_conv_first_fwd: stride %d", stride);
  PO_REQUIRE(Cout > 0 && Cout <= 64 && Cout_p % 4 == 0 && Cout_p >= Cout, "po_conv_first_fwd: Cout=%d Cout_p=%d", Cout, Cout_p);
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const int64_t n = (int64_t)B * Ho * Wo;
  dim3 grid(po::ceil_div(n, 256));
  hipStream_t st = po::stream_of(s);
  const int CO = Cout_p <= 16 ? 16 : (Cout_p <= 32 ? 32 : 64);
  PO_REQUIRE(Cout_p == CO, "po_conv_first_fwd: Cout_p must be 16, 32 or 64 (got %d)", Cout_p);
  if (CO == 16)
    hipLaunchKernelGGL(first_fwd_k<16>, grid, dim3(256), 0, st, img, B, H, W, stride, Ho, Wo, Wt, bias, Cout, Cout_p, act, y);
  else if (CO == 32)
    hipLaunchKernelGGL(first_fwd_k<32>, grid, dim3(256), 0, st, img, B, H, W, stride, Ho, Wo, Wt, bias, Cout, Cout_p, act, y);
  else
    hipLaunchKernelGGL(first_fwd_k<64>, grid, dim3(256), 0, st, img, B, H, W, stride, Ho, Wo, Wt, bias, Cout, Cout_p, act, y);
  return po::check_launch("po_conv_first_fwd");
}

extern "C" int po_conv_first_dgrad(const float* D, int B, int H, int W, int stride, const float* Wt,
                                   int Cout, int Cout_p, float* d_img, po_stream_t s) {
  PO_REQUIRE(D && Wt && d_img, "po_conv_first_dgrad: null pointer");
  PO_REQUIRE(stride == 1 || stride == 2, "po_conv_first_dgrad: stride %d", stride);
  const int CO = Cout_p <= 16 ? 16 : (Cout_p <= 32 ? 32 : 64);
  PO_REQUIRE(Cout_p == CO && Cout <= Cout_p, "po_conv_first_dgrad: Cout_p must be 16, 32 or 64 (got %d)", Cout_p);
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const int64_t n = (int64_t)B * H * W;
  dim3 grid(po::ceil_div(n, 256));
  hipStream_t st = po::stream_of(s);
  if (CO == 16)
    hipLaunchKernelGGL(first_dgrad_k<16>, grid, dim3(256), 0, st, D, B, H, W, stride, Ho, Wo, Wt, Cout, Cout_p, d_img);
  else if (CO == 32)
    hipLaunchKernelGGL(first_dgrad_k<32>, grid, dim3(256), 0, st, D, B, H, W, stride, Ho, Wo, Wt, Cout, Cout_p, d_img);
  else
    hipLaunchKernelGGL(first_dgrad_k<64>, grid, dim3(256), 0, st, D, B, H, W, stride, Ho, Wo, Wt, Cout, Cout_p, d_img);
  return po::check_launch("po_conv_first_dgrad");
}
