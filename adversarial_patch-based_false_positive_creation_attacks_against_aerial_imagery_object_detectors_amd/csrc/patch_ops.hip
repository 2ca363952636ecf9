// Patch-side kernels for gfx950: median pool, placement parameters, the fused
// augment + affine-warp + composite (forward and deterministic gather-form
// backward), PatchApplier, and the NPS/TV/colour regularisers.
//
// Float operation order follows the reference's PyTorch ops (no FMA
// contraction in this file) so the exact-zero composite test and the clamp
// masks route gradients like the reference.
#pragma clang fp contract(off)
#include "common.h"
#include "philox.h"
#include "warp_geom.h"
#include <math.h>
#include <string.h>
#include <algorithm>

namespace po {
static thread_local char g_err[512] = {0};
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace po

extern "C" int po_abi_version(void) { return PO_ABI_VERSION; }
extern "C" const char* po_last_error(void) { return po::g_err; }

extern "C" int po_device_check(int device) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    po::set_error("hipSetDevice(%d): %s", device, hipGetErrorString(e));
    return PO_EHIP;
  }
  hipDeviceProp_t p;
  e = hipGetDeviceProperties(&p, device);
  if (e != hipSuccess) {
    po::set_error("hipGetDeviceProperties: %s", hipGetErrorString(e));
    return PO_EHIP;
  }
  if (strncmp(p.gcnArchName, "gfx950", 6) != 0) {
    po::set_error("device %d is %s, this library is built for gfx950 only", device, p.gcnArchName);
    return PO_EDEVICE;
  }
  return PO_OK;
}

// ------------------------------------------------------------------------
// Median pool 7x7, reflect padding (median_pool.py:26-52)
// ------------------------------------------------------------------------
namespace {
constexpr int MT = 16;             // output tile
constexpr int MH = MT + 6;         // input tile with halo

__device__ __forceinline__ int reflect_idx(int k, int n) {
  return k < 0 ? -k : (k >= n ? 2 * (n - 1) - k : k);
}

__global__ __launch_bounds__(256) void median7_fwd_k(const float* __restrict__ x, int H, int W,
                                                     float* __restrict__ y, int32_t* __restrict__ arg) {
  __shared__ float tile[MH][MH + 1];
  const int c = blockIdx.z, i0 = blockIdx.y * MT, j0 = blockIdx.x * MT;
  const float* xc = x + (size_t)c * H * W;
  for (int t = threadIdx.x; t < MH * MH; t += 256) {
    int ti = t / MH, tj = t % MH;
    int r = reflect_idx(min(max(i0 + ti - 3, -3), H + 2), H);
    int q = reflect_idx(min(max(j0 + tj - 3, -3), W + 2), W);
    tile[ti][tj] = xc[(size_t)r * W + q];
  }
  __syncthreads();
  const int ty = threadIdx.x / MT, tx = threadIdx.x % MT;
  const int i = i0 + ty, j = j0 + tx;
  if (i >= H || j >= W) return;
  float v[49];
  bool nan = false;
#pragma unroll
  for (int a = 0; a < 49; ++a) {
    v[a] = tile[ty + a / 7][tx + a % 7];
    nan |= v[a] != v[a];
  }
  // the 25th smallest (index 24) of 49; the argument is the first window
  // position (row-major) holding the median value.
  int found = 48;
  if (!nan) {
    // a bitonic sort of the 49 values padded to 64 with +inf (672 min/max
    // pairs in registers) gives the value; the first position holding it is
    // the rank-counting rule's argument (any position whose value equals the
    // 25th smallest has < 25 smaller and >= 25 not-larger values; -0 and +0
    // compare equal, as in the counting)
    float srt[64];
#pragma unroll
    for (int a = 0; a < 64; ++a) srt[a] = a < 49 ? v[a] : INFINITY;
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
      for (int jj = k >> 1; jj > 0; jj >>= 1)
#pragma unroll
        for (int a = 0; a < 64; ++a) {
          const int l = a ^ jj;
          if (l > a) {
            const float lo = fminf(srt[a], srt[l]), hi = fmaxf(srt[a], srt[l]);
            const bool up = (a & k) == 0;
            srt[a] = up ? lo : hi;
            srt[l] = up ? hi : lo;
          }
        }
    const float m24 = srt[24];
#pragma unroll
    for (int a = 48; a >= 0; --a)
      if (v[a] == m24) found = a;
  } else {
    // rank selection by counting (NaN compares false, as in the reference's sort)
#pragma unroll 1
    for (int a = 48; a >= 0; --a) {
      int less = 0, leq = 0;
#pragma unroll
      for (int b = 0; b < 49; ++b) {
        less += v[b] < v[a];
        leq += v[b] <= v[a];
      }
      if (less <= 24 && leq > 24) found = a;
    }
  }
  float med = v[0];
#pragma unroll
  for (int a = 0; a < 49; ++a) med = (a == found) ? v[a] : med;
  const int di = found / 7, dj = found % 7;
  const int r = reflect_idx(i + di - 3, H), q = reflect_idx(j + dj - 3, W);
  y[(size_t)c * H * W + (size_t)i * W + j] = med;
  arg[(size_t)c * H * W + (size_t)i * W + j] = (int32_t)((size_t)c * H * W + (size_t)r * W + q);
}

// dx[p] = sum over outputs o within the 7x7 neighbourhood of p with
// argidx[o] == p (reflection images of p fall inside that neighbourhood).
__global__ __launch_bounds__(256) void median7_bwd_k(const float* __restrict__ dy,
                                                     const int32_t* __restrict__ arg, int C, int H,
                                                     int W, float* __restrict__ dx) {
  const int64_t n = (int64_t)C * H * W;
  int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= n) return;
  const int c = (int)(p / ((int64_t)H * W));
  const int rem = (int)(p - (int64_t)c * H * W);
  const int r = rem / W, q = rem % W;
  const size_t base = (size_t)c * H * W;
  float acc = 0.f;
  for (int i = max(0, r - 3); i <= min(H - 1, r + 3); ++i)
    for (int j = max(0, q - 3); j <= min(W - 1, q + 3); ++j) {
      size_t o = base + (size_t)i * W + j;
      if (arg[o] == (int32_t)p) acc += dy[o];
    }
  dx[p] = acc;
}
}  // namespace

extern "C" int po_median7_fwd(const float* x, int C, int H, int W, float* y, int32_t* argidx,
                              po_stream_t s) {
  PO_REQUIRE(x && y && argidx, "po_median7_fwd: null pointer");
  PO_REQUIRE(C > 0 && H > 3 && W > 3, "po_median7_fwd: need C>0, H>3, W>3 (reflect pad 3), got %d %d %d", C, H, W);
  dim3 grid(po::ceil_div(W, MT), po::ceil_div(H, MT), C);
  hipLaunchKernelGGL(median7_fwd_k, grid, dim3(256), 0, po::stream_of(s), x, H, W, y, argidx);
  return po::check_launch("po_median7_fwd");
}

extern "C" int po_median7_bwd(const float* dy, const int32_t* argidx, int C, int H, int W, float* dx,
                              po_stream_t s) {
  PO_REQUIRE(dy && argidx && dx, "po_median7_bwd: null pointer");
  PO_REQUIRE(C > 0 && H > 3 && W > 3, "po_median7_bwd: bad shape");
  int64_t n = (int64_t)C * H * W;
  hipLaunchKernelGGL(median7_bwd_k, dim3(po::ceil_div(n, 256)), dim3(256), 0, po::stream_of(s), dy,
                     argidx, C, H, W, dx);
  return po::check_launch("po_median7_bwd");
}

// ------------------------------------------------------------------------
// General median pool (median_pool.py:8-52 for any kernel, stride and
// padding): reflect pad (l, r, t, b), kh x kw windows at stride (sh, sw), the
// lower median (torch.median: rank (n-1)/2), argument = the first window
// position (row-major) holding it.  Not on the training path (the patch
// transformer uses the 7x7 kernels above); rank by counting, O(n^2) per
// output from the L1/L2-resident plane.
// ------------------------------------------------------------------------
namespace {
struct MedGeom {
  int H, W, kh, kw, sh, sw, pl, pt, Ho, Wo;
};

__global__ __launch_bounds__(256) void median_fwd_k(const float* __restrict__ x, int C, MedGeom g,
                                                    float* __restrict__ y, int32_t* __restrict__ arg) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= (int64_t)C * g.Ho * g.Wo) return;
  const int c = (int)(q / ((int64_t)g.Ho * g.Wo));
  const int rem = (int)(q - (int64_t)c * g.Ho * g.Wo);
  const int i = rem / g.Wo, j = rem - (rem / g.Wo) * g.Wo;
  const float* xc = x + (size_t)c * g.H * g.W;
  const int n = g.kh * g.kw, r = (n - 1) / 2;
  auto val = [&](int a) {
    const int rr = reflect_idx(i * g.sh + a / g.kw - g.pt, g.H), cc = reflect_idx(j * g.sw + a % g.kw - g.pl, g.W);
    return xc[(size_t)rr * g.W + cc];
  };
  int found = 0;
  float med = 0.f;
  for (int a = 0; a < n; ++a) {
    const float va = val(a);
    int less = 0, leq = 0;
    for (int b2 = 0; b2 < n; ++b2) {
      const float vb = val(b2);
      less += vb < va;
      leq += vb <= va;
    }
    if (less <= r && leq > r) { found = a; med = va; break; }     // first position holding the median
  }
  const int rr = reflect_idx(i * g.sh + found / g.kw - g.pt, g.H), cc = reflect_idx(j * g.sw + found % g.kw - g.pl, g.W);
  y[q] = med;
  arg[q] = (int32_t)((size_t)c * g.H * g.W + (size_t)rr * g.W + cc);
}

// dx[p] = sum, in output order, of dy[o] over the outputs o whose argument
// is p.  Candidate outputs: those whose window covers one of the padded
// positions reflecting onto p's row and column (up to 3 each); each output is
// visited once (the union of the ranges is scanned), so a window holding two
// reflections of p still routes its gradient once, as torch's unfold + pad
// backward does.
__global__ __launch_bounds__(256) void median_bwd_k(const float* __restrict__ dy, const int32_t* __restrict__ arg,
                                                    int C, MedGeom g, int pb, int pr, float* __restrict__ dx) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= (int64_t)C * g.H * g.W) return;
  const int c = (int)(p / ((int64_t)g.H * g.W));
  const int rem = (int)(p - (int64_t)c * g.H * g.W);
  const int r0 = rem / g.W, c0 = rem - (rem / g.W) * g.W;
  // padded coordinates (from the padded origin) that reflect onto r0 / c0
  int us[3], nu = 0, vs[3], nv = 0;
  us[nu++] = r0 + g.pt;
  if (r0 > 0 && r0 <= g.pt) us[nu++] = g.pt - r0;                                   // u = -r0
  if (r0 < g.H - 1 && g.H - 1 - r0 <= pb) us[nu++] = 2 * (g.H - 1) - r0 + g.pt;     // u = 2(H-1) - r0
  vs[nv++] = c0 + g.pl;
  if (c0 > 0 && c0 <= g.pl) vs[nv++] = g.pl - c0;
  if (c0 < g.W - 1 && g.W - 1 - c0 <= pr) vs[nv++] = 2 * (g.W - 1) - c0 + g.pl;
  int i0 = g.Ho, i1 = -1, j0 = g.Wo, j1 = -1;
  for (int a = 0; a < nu; ++a) {
    i0 = min(i0, max(0, (us[a] - g.kh + g.sh) / g.sh));
    i1 = max(i1, min(g.Ho - 1, us[a] / g.sh));
  }
  for (int b = 0; b < nv; ++b) {
    j0 = min(j0, max(0, (vs[b] - g.kw + g.sw) / g.sw));
    j1 = max(j1, min(g.Wo - 1, vs[b] / g.sw));
  }
  const int32_t want = (int32_t)p;
  const size_t base = (size_t)c * g.Ho * g.Wo;
  float acc = 0.f;
  for (int i = i0; i <= i1; ++i)
    for (int j = j0; j <= j1; ++j)
      if (arg[base + (size_t)i * g.Wo + j] == want) acc += dy[base + (size_t)i * g.Wo + j];
  dx[p] = acc;
}
}  // namespace

extern "C" int po_median_fwd(const float* x, int C, int H, int W, int kh, int kw, int sh, int sw, int pl, int pr,
                             int pt, int pb, float* y, int32_t* argidx, po_stream_t s) {
  PO_REQUIRE(x && y && argidx, "po_median_fwd: null pointer");
  PO_REQUIRE(C > 0 && H > 0 && W > 0 && kh > 0 && kw > 0 && sh > 0 && sw > 0, "po_median_fwd: bad shape");
  PO_REQUIRE(kh * kw <= 1024, "po_median_fwd: window of %d elements (max 1024)", kh * kw);
  PO_REQUIRE(pl >= 0 && pr >= 0 && pt >= 0 && pb >= 0 && pl < W && pr < W && pt < H && pb < H,
             "po_median_fwd: reflect padding must be smaller than the input (F.pad mode='reflect')");
  const int Hp = H + pt + pb, Wp = W + pl + pr;
  PO_REQUIRE(Hp >= kh && Wp >= kw, "po_median_fwd: window larger than the padded input");
  MedGeom g{H, W, kh, kw, sh, sw, pl, pt, (Hp - kh) / sh + 1, (Wp - kw) / sw + 1};
  const int64_t n = (int64_t)C * g.Ho * g.Wo;
  hipLaunchKernelGGL(median_fwd_k, dim3(po::ceil_div(n, 256)), dim3(256), 0, po::stream_of(s), x, C, g, y, argidx);
  return po::check_launch("po_median_fwd");
}

extern "C" int po_median_bwd(const float* dy, const int32_t* argidx, int C, int H, int W, int kh, int kw, int sh,
                             int sw, int pl, int pr, int pt, int pb, float* dx, po_stream_t s) {
  PO_REQUIRE(dy && argidx && dx, "po_median_bwd: null pointer");
  PO_REQUIRE(C > 0 && H > 0 && W > 0 && kh > 0 && kw > 0 && sh > 0 && sw > 0 && pl >= 0 && pr >= 0 && pt >= 0 &&
                 pb >= 0 && pl < W && pr < W && pt < H && pb < H,
             "po_median_bwd: bad shape");
  const int Hp = H + pt + pb, Wp = W + pl + pr;
  PO_REQUIRE(Hp >= kh && Wp >= kw, "po_median_bwd: window larger than the padded input");
  MedGeom g{H, W, kh, kw, sh, sw, pl, pt, (Hp - kh) / sh + 1, (Wp - kw) / sw + 1};
  const int64_t n = (int64_t)C * H * W;
  hipLaunchKernelGGL(median_bwd_k, dim3(po::ceil_div(n, 256)), dim3(256), 0, po::stream_of(s), dy, argidx, C, g,
                     pb, pr, dx);
  return po::check_launch("po_median_bwd");
}

// ------------------------------------------------------------------------
// Placement parameters (load_data.py:453-509, 654-743)
// ------------------------------------------------------------------------
namespace {
constexpr float kDrawPi = 3.14159265358979323846f;   // po_draws' pi (draw_ops.hip)
constexpr int kLatticeN = 1 << 24;

// sin and cos of an angle as torch.sin / torch.cos compute them on the CPU
// (load_data.py:731-732; MKL VML, not correctly rounded, so not restatable):
// angles on po_draws' lattice (angle_k = fp32(k 2^-24 fp32(2 pi) - pi)) are
// looked up in `lut` [2^24][2] (load_data.sincos_lattice_table: the CPU's own
// values, tabulated once per process); any other angle, or no table, gets the
// correctly rounded values (float64 evaluation rounded once), which equal
// the CPU's in ~95 % of cases.
__device__ __forceinline__ void ref_sincos(float a, const float* __restrict__ lut, float& sn, float& cs) {
  if (lut) {
    const double span = (double)(2.0f * kDrawPi), from = (double)(-kDrawPi);
    const double kd = rint(((double)a - from) / span * 16777216.0);
    if (kd >= -1.0 && kd <= 16777216.0) {
      const int k0 = (int)kd;
      for (int d = -1; d <= 1; ++d) {
        const int k = k0 + d;
        if (k < 0 || k >= kLatticeN) continue;
        const float ak = (float)((double)((float)k * 0x1p-24f) * span + from);
        if (__float_as_uint(ak) == __float_as_uint(a)) {
          const float2 v = reinterpret_cast<const float2*>(lut)[k];
          sn = v.x;
          cs = v.y;
          return;
        }
      }
    }
  }
  sn = (float)sin((double)a);
  cs = (float)cos((double)a);
}

// sqrt of a target size's square as torch.sqrt computes it on the CPU
// (load_data.py:667-668; MKL VML's vsSqrt, not correctly rounded: ~0.6 % of
// values one ulp off on Intel AVX-512, ~17 % on the AMD EPYC hosts of the
// MI355X boxes).  Its result scales exactly with the input's powers of 4
// (sqrt(4^k m) = 2^k sqrt(m), measured: tests/test_geometry_ref.py), so
// `lut` holds the host's values over one period, m in [1, 4) (2^24 floats,
// entry i = sqrt of the float with bits 0x3F800000 + i;
// load_data.sqrt_period_table); a normal positive v = 4^k m reads entry
// (exponent parity, mantissa) and scales by 2^k.  No table, or zero, a
// subnormal, inf or NaN: the correctly rounded value.
__device__ __forceinline__ float ref_sqrt(float v, const float* __restrict__ lut) {
  const uint32_t u = __float_as_uint(v);
  const int e = (int)((u >> 23) & 0xff);
  if (!lut || (u >> 31) || e == 0 || e == 0xff) return sqrtf(v);      // correctly rounded (HIP default)
  const int ue = e - 127;                                     // v = 2^ue * 1.f
  const int k = ue >= 0 ? ue / 2 : -((1 - ue) / 2);           // floor(ue / 2)
  const uint32_t idx = ((uint32_t)(ue - 2 * k) << 23) | (u & 0x7fffffu);   // m = 4^-k v in [1, 4)
  return __builtin_ldexpf(lut[idx], k);
}

// one wave per image: the label scan is a wave reduction of (area, row) pairs
__global__ __launch_bounds__(64) void patch_params_k(const float* __restrict__ lab, int B, int L,
                                                     const float* __restrict__ angle, const float* __restrict__ ux,
                                                     const float* __restrict__ uy, int do_rotate, int S, int P,
                                                     int geometry, const float* __restrict__ lut,
                                                     const float* __restrict__ sqrt_lut,
                                                     float* __restrict__ theta, float* __restrict__ center,
                                                     float* __restrict__ tsize, int32_t* __restrict__ roi,
                                                     double* __restrict__ affine) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const float* lb = lab + (size_t)b * L * 5;
  // lab_transform: area = lab[:,:,3]*lab[:,:,4]; torch.max / torch.min over
  // rows, first index on ties (load_data.py:464-467)
  float vmax = -INFINITY, vmin = INFINITY;
  int imax = 0x7fffffff, imin = 0x7fffffff;
  for (int l = lane; l < L; l += 64) {
    float a = lb[l * 5 + 3] * lb[l * 5 + 4];
    if (a > vmax) { vmax = a; imax = l; }
    if (a < vmin) { vmin = a; imin = l; }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(vmax, o), nv = __shfl_xor(vmin, o);
    const int oi = __shfl_xor(imax, o), ni = __shfl_xor(imin, o);
    if (ov > vmax || (ov == vmax && oi < imax)) { vmax = ov; imax = oi; }
    if (nv < vmin || (nv == vmin && ni < imin)) { vmin = nv; imin = ni; }
  }
  if (lane != 0) return;
  // patch centre in fp32 exactly as the reference (load_data.py:703-715): the
  // loss cell index is derived from it and must be bit-exact
  const float fS = (float)S;
  const float tx_f = fmaxf(ux[b], 0.2f);     // load_data.py:703
  const float ty_f = fminf(uy[b], 0.8f);     // load_data.py:706
  center[2 * b + 0] = tx_f * fS;             // load_data.py:712-715
  center[2 * b + 1] = ty_f * fS;
  if (geometry == 1 || geometry == 2) {
    // the reference's fp32 arithmetic, op by op (warp_geom.h): lab_transform's
    // (max row + min row) / 2 (load_data.py:474-477), * img_size (654-660),
    // .mul(1/2) ** 2, the sum and sqrt (667-668), / patch side (717)
    float s2 = 0.25f, s3 = 0.25f;
    if (!(vmax > 0.99f)) {
      s2 = (lb[imax * 5 + 2] + lb[imin * 5 + 2]) / 2.0f;
      s3 = (lb[imax * 5 + 3] + lb[imin * 5 + 3]) / 2.0f;
    }
    // (this file: fp contract(off) -- every operator below is one rounding)
    const float h2 = (s2 * fS) * 0.5f, h3 = (s3 * fS) * 0.5f;
    const float ts = ref_sqrt(h2 * h2 + h3 * h3, sqrt_lut);
    const float sc = ts / (float)P;
    const float tx = (-tx_f + 0.5f) * 2.0f;                               // load_data.py:726
    const float ty = (-ty_f + 0.5f) * 2.0f;                               // load_data.py:727
    float sn = 0.f, cs = 1.f;                                              // angle fill_(0): 614
    if (do_rotate) ref_sincos(angle[b], lut, sn, cs);
    float th[6];
    po::ref_theta(sn, cs, sc, tx, ty, th);
    float* tho = theta + 6 * b;
    for (int k = 0; k < 6; ++k) tho[k] = th[k];
    if (tsize) tsize[b] = ts;
    if (affine) po::store_ref_row(th, geometry, affine + 6 * b);
    if (roi) {
      double thd[6], af[6];
      for (int k = 0; k < 6; ++k) thd[k] = (double)th[k];
      po::theta_pixel_affine(thd, (double)S, af);
      po::footprint_roi(af, S, P, roi + 4 * b);
    }
    return;
  }
  // Placement geometry in float64 (from the same fp32 labels and draws).  The
  // translation terms of theta reach |tx cos / scale| ~ 10-20 and cancel in the
  // affine grid down to the patch's ~0.4; in fp32 that cancellation leaves
  // ~1e-4 px of error in the sampling coordinates, i.e. ~1e-4 relative in the
  // bilinear weights and the patch gradient.  In double the HIP warp samples
  // where the exact (float64) evaluation of the reference formulas samples.
  double sel2, sel3;
  if (vmax > 0.99f) {                        // load_data.py:471-473
    sel2 = 0.25; sel3 = 0.25;
  } else {                                   // load_data.py:474-477
    sel2 = ((double)lb[imax * 5 + 2] + (double)lb[imin * 5 + 2]) / 2.0;
    sel3 = ((double)lb[imax * 5 + 3] + (double)lb[imin * 5 + 3]) / 2.0;
  }
  const double dS = (double)S;
  const double h2 = sel2 * dS * 0.5, h3 = sel3 * dS * 0.5;   // load_data.py:651-655, 1/SCALE_FACTOR
  const double ts = sqrt(h2 * h2 + h3 * h3);                 // load_data.py:662-663
  const double txd = fmax((double)ux[b], 0.2), tyd = fmin((double)uy[b], 0.8);
  const double scale = ts / (double)P;                       // load_data.py:717
  const double tx = (-txd + 0.5) * 2.0;                      // load_data.py:726
  const double ty = (-tyd + 0.5) * 2.0;                      // load_data.py:727
  const double a = do_rotate ? (double)angle[b] : 0.0;
  double th[6], af[6];
  po::placement_theta(a, scale, tx, ty, th);                   // load_data.py:738-743
  float* tho = theta + 6 * b;
  for (int k = 0; k < 6; ++k) tho[k] = (float)th[k];
  if (tsize) tsize[b] = (float)ts;
  po::theta_pixel_affine(th, dS, af);
  if (affine)
    for (int k = 0; k < 6; ++k) affine[6 * b + k] = af[k];
  if (roi) po::footprint_roi(af, S, P, roi + 4 * b);
}
}  // namespace

extern "C" int po_patch_params(const float* lab, int B, int L, const float* angle, const float* ux,
                               const float* uy, int do_rotate, int S, int P, int geometry,
                               const float* sincos_lut, const float* sqrt_lut, float* theta, float* center,
                               float* target_size, int32_t* roi, double* affine, po_stream_t s) {
  PO_REQUIRE(lab && ux && uy && theta && center, "po_patch_params: null pointer");
  PO_REQUIRE(!do_rotate || angle, "po_patch_params: angle required when do_rotate");
  PO_REQUIRE(B > 0 && L > 0 && S > 0 && P > 0, "po_patch_params: bad shape");
  PO_REQUIRE(geometry == 0 || ((geometry == 1 || geometry == 2) && S > 1),
             "po_patch_params: geometry must be 0 (float64), 1 or 2 (reference fp32, S > 1)");
  PO_REQUIRE(!sincos_lut || ((uintptr_t)sincos_lut % 8) == 0, "po_patch_params: sincos_lut must be 8-byte aligned");
  hipLaunchKernelGGL(patch_params_k, dim3(B), dim3(64), 0, po::stream_of(s), lab, B, L, angle, ux, uy,
                     do_rotate, S, P, geometry, sincos_lut, sqrt_lut, theta, center, target_size, roi, affine);
  return po::check_launch("po_patch_params");
}

// ------------------------------------------------------------------------
// Augment + affine warp + clamp*mask (+ composite)  (load_data.py:548-792, 820)
// ------------------------------------------------------------------------
namespace {
struct WarpGeom {
  int S, P, padL, padT;
  // noise key (po_warp_*_keyed): with no noise tensor the kernels regenerate
  // element e of image b as po_draws does (philox_noise, global image nb0 + b)
  uint32_t nk0, nk1, nc_lo, nc_hi;
  int nb0;
  // pre-augmented patches (po_warp_*_pre): [B][3][P][P] values mp*contrast +
  // bright + 0.1*noise before the clamp (po_augment_patch); the kernels then
  // read them instead of forming them from mp, the draws and the noise
  const float* pre;
  po::RefAxis ax;        // the reference geometry's per-axis constants (po::ref_axis(S))
};

// The transformer noise of one image: the explicit tensor [3][P][P], or (nz
// NULL) regenerated in-kernel from the po_draws key — bit-identical values,
// without the B*3*P*P*4-byte noise tensor being written and gathered.
struct NoiseSrc {
  const float* nz;
  const float* pre;       // this image's pre-augmented values, or NULL
  uint32_t k0, k1, c_lo, c_hi, gb;
  __device__ __forceinline__ float at(size_t e) const {
    return nz ? nz[e] : po::philox_noise(k0, k1, c_lo, c_hi, gb, (uint32_t)e);
  }
};
__device__ __forceinline__ NoiseSrc noise_src(const float* noise, const WarpGeom& g, int b) {
  NoiseSrc ns;
  ns.nz = noise ? noise + (size_t)b * 3 * g.P * g.P : nullptr;
  ns.pre = g.pre ? g.pre + (size_t)b * 3 * g.P * g.P : nullptr;
  ns.k0 = g.nk0; ns.k1 = g.nk1; ns.c_lo = g.nc_lo; ns.c_hi = g.nc_hi;
  ns.gb = (uint32_t)(g.nb0 + b);
  return ns;
}

// Source coordinate (ix: column, iy: row) in the padded patch of output pixel
// (i, j): affine_grid (align_corners=False) + grid_sampler_unnormalize folded
// into the pixel-space affine af (po_patch_params), evaluated in float64.
__device__ __forceinline__ void sample_coord(const double* af, int i, int j, double& ix, double& iy) {
  ix = fma(af[0], (double)j, fma(af[1], (double)i, af[2]));
  iy = fma(af[3], (double)j, fma(af[4], (double)i, af[5]));
}

// Bilinear corner (x0, y0) and weights {nw, ne, sw, se} of a sample point
// (weights from the float64 coordinate, rounded once to fp32)
__device__ __forceinline__ void bilinear(double ix, double iy, int& x0, int& y0, float w[4]) {
  const double fx = floor(ix), fy = floor(iy);
  x0 = (int)fx;
  y0 = (int)fy;
  const double ex = ix - fx, ey = iy - fy;              // in [0, 1)
  w[0] = (float)((1.0 - ex) * (1.0 - ey));
  w[1] = (float)(ex * (1.0 - ey));
  w[2] = (float)((1.0 - ex) * ey);
  w[3] = (float)(ex * ey);
}

// The bilinear corner (x0, y0) and weights {nw, ne, sw, se} of output pixel
// (i, j) under image geometry G; false if no corner lies in the padded patch
// region [pad - 1, pad + P) -- the output is then exactly 0.  Reference form:
// grid_sample's fp32 arithmetic (warp_geom.h; GridSamplerKernel.cpp: w = ix -
// floor(ix), e = 1 - w, nw = s*e, ne = s*w, sw = n*e, se = n*w).
__device__ __forceinline__ bool sample_point_ref(const float th[6], int form, const WarpGeom& g, int i, int j,
                                                 int& x0, int& y0, float w[4]) {
  float ix, iy;
  po::ref_sample_coord(th, form, g.ax, i, j, ix, iy);
  if (!(ix >= (float)(g.padL - 1) && ix < (float)(g.padL + g.P) && iy >= (float)(g.padT - 1) &&
        iy < (float)(g.padT + g.P)))
    return false;
  const float fx = floorf(ix), fy = floorf(iy);
  x0 = (int)fx;
  y0 = (int)fy;
  const float ex = ix - fx, wx = 1.0f - ex;          // (file-wide fp contract(off))
  const float ny = iy - fy, sy = 1.0f - ny;
  w[0] = sy * wx;
  w[1] = sy * ex;
  w[2] = ny * wx;
  w[3] = ny * ex;
  return true;
}
__device__ __forceinline__ bool sample_point_f64(const double af[6], const WarpGeom& g, int i, int j, int& x0,
                                                 int& y0, float w[4]) {
  double ix, iy;
  sample_coord(af, i, j, ix, iy);
  if (!(ix >= (double)(g.padL - 1) && ix < (double)(g.padL + g.P) && iy >= (double)(g.padT - 1) &&
        iy < (double)(g.padT + g.P)))
    return false;
  bilinear(ix, iy, x0, y0, w);
  return true;
}
__device__ __forceinline__ bool sample_point(const po::Geo& G, const WarpGeom& g, int i, int j, int& x0, int& y0,
                                             float w[4]) {
  return G.ref ? sample_point_ref(G.th, G.ref, g, i, j, x0, y0, w) : sample_point_f64(G.af, g, i, j, x0, y0, w);
}

__device__ __forceinline__ float aug_value(const float* __restrict__ mp, const NoiseSrc& ns,
                                           float contrast, float bright, int ch, int pr, int pc, int P) {
  const size_t o = ((size_t)ch * P + pr) * P + pc;
  const float v = ns.pre ? ns.pre[o] : mp[o] * contrast + bright + ns.at(o) * 0.1f;    // load_data.py:566-571
  return fminf(fmaxf(v, 0.f), 1.f);                      // load_data.py:574
}

// one bilinear term: the reference form accumulates as grid_sample's fma
// chain (fma(v, w, acc) corner after corner), the float64 form adds products
__device__ __forceinline__ float bterm(bool ref, float v, float w, float acc) {
  return ref ? __builtin_fmaf(v, w, acc) : acc + v * w;
}

// Forward of one output pixel: adv_t[3] (clamped) and msk_t.  Returns false
// if no neighbour lies inside the padded patch region (output exactly 0).
template <bool AUG = true>
__device__ __forceinline__ bool warp_pixel(const po::Geo& G, const WarpGeom& g, const float* mp,
                                           const NoiseSrc& nz, float contrast, float bright, int i, int j,
                                           float adv[3], float& msk, bool raw_in_range[3]) {
  int x0, y0;
  float w[4];
  if (!sample_point(G, g, i, j, x0, y0, w)) return false;
  const bool ref = G.ref != 0;
  const int cx[4] = {x0, x0 + 1, x0, x0 + 1};
  const int cy[4] = {y0, y0, y0 + 1, y0 + 1};
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, m = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int pr = cy[k] - g.padT, pc = cx[k] - g.padL;
    if (pr >= 0 && pr < g.P && pc >= 0 && pc < g.P) {
      if (AUG) {
        a0 = bterm(ref, aug_value(mp, nz, contrast, bright, 0, pr, pc, g.P), w[k], a0);
        a1 = bterm(ref, aug_value(mp, nz, contrast, bright, 1, pr, pc, g.P), w[k], a1);
        a2 = bterm(ref, aug_value(mp, nz, contrast, bright, 2, pr, pc, g.P), w[k], a2);
      } else {                                // test_real: clamp(patch) only (load_data.py:1070-1076)
        const size_t o = (size_t)pr * g.P + pc, pp = (size_t)g.P * g.P;
        a0 = bterm(ref, fminf(fmaxf(mp[o], 0.f), 1.f), w[k], a0);
        a1 = bterm(ref, fminf(fmaxf(mp[o + pp], 0.f), 1.f), w[k], a1);
        a2 = bterm(ref, fminf(fmaxf(mp[o + 2 * pp], 0.f), 1.f), w[k], a2);
      }
      m = bterm(ref, 1.f, w[k], m);
    }
  }
  raw_in_range[0] = a0 >= 0.f && a0 <= 1.f;
  raw_in_range[1] = a1 >= 0.f && a1 <= 1.f;
  raw_in_range[2] = a2 >= 0.f && a2 <= 1.f;
  adv[0] = fminf(fmaxf(a0, 0.f), 1.f);
  adv[1] = fminf(fmaxf(a1, 0.f), 1.f);
  adv[2] = fminf(fmaxf(a2, 0.f), 1.f);
  msk = m;
  return true;
}

__global__ __launch_bounds__(256) void warp_fwd_k(const float* __restrict__ img,
                                                  const float* __restrict__ mp,
                                                  const float* __restrict__ noise,
                                                  const float* __restrict__ contrast,
                                                  const float* __restrict__ bright,
                                                  const double* __restrict__ affine, WarpGeom g, int mode,
                                                  float* __restrict__ out) {
  const int b = blockIdx.z;
  const int i = blockIdx.y, j = blockIdx.x * 256 + threadIdx.x;
  if (j >= g.S) return;
  const size_t plane = (size_t)g.S * g.S;
  const size_t o = (size_t)b * 3 * plane + (size_t)i * g.S + j;
  float adv[3], msk;
  bool rng[3];
  const po::Geo G = po::load_geo(affine + 6 * b, g.S);
  const bool hit = warp_pixel(G, g, mp, noise_src(noise, g, b), g.pre ? 1.f : contrast[b],
                              g.pre ? 0.f : bright[b], i, j, adv, msk, rng);
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    float v = hit ? adv[ch] * msk : 0.f;          // load_data.py:791-792
    if (mode == 1) v = (v == 0.f) ? img[o + ch * plane] : v;   // load_data.py:820
    out[o + ch * plane] = v;
  }
}

// Four consecutive pixels of a row per thread (S % 4 == 0): the same
// per-pixel arithmetic as warp_fwd_k, with 16-byte image reads and output
// writes, threads laid over the image's (row, pixel quad) grid.
__global__ __launch_bounds__(256) void warp_fwd4_k(const float* __restrict__ img,
                                                   const float* __restrict__ mp,
                                                   const float* __restrict__ noise,
                                                   const float* __restrict__ contrast,
                                                   const float* __restrict__ bright,
                                                   const double* __restrict__ affine, WarpGeom g, int mode,
                                                   float* __restrict__ out) {
  const int b = blockIdx.y;
  const int sq = g.S >> 2;
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= g.S * sq) return;
  const int i = q / sq, j0 = (q - i * sq) * 4;
  const size_t plane = (size_t)g.S * g.S;
  const size_t o = (size_t)b * 3 * plane + (size_t)i * g.S + j0;
  const po::Geo G = po::load_geo(affine + 6 * b, g.S);
  const NoiseSrc nz = noise_src(noise, g, b);
  const float cb = g.pre ? 1.f : contrast[b], bb = g.pre ? 0.f : bright[b];
  float v[3][4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    float adv[3], msk;
    bool rng[3];
    const bool hit = warp_pixel(G, g, mp, nz, cb, bb, i, j0 + u, adv, msk, rng);
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) v[ch][u] = hit ? adv[ch] * msk : 0.f;   // load_data.py:791-792
  }
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    if (mode == 1) {                                                       // load_data.py:820
      const float4 m = *reinterpret_cast<const float4*>(img + o + ch * plane);
      const float mv[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) v[ch][u] = (v[ch][u] == 0.f) ? mv[u] : v[ch][u];
    }
    *reinterpret_cast<float4*>(out + o + ch * plane) = make_float4(v[ch][0], v[ch][1], v[ch][2], v[ch][3]);
  }
}

// Backward phase A: per output pixel of the footprint,
// gfac = d_out * [out != 0 (mode 1)] * msk_t * [0 <= adv_t <= 1]
__global__ __launch_bounds__(256) void warp_bwd_a_k(const float* __restrict__ d_out,
                                                    const float* __restrict__ mp,
                                                    const float* __restrict__ noise,
                                                    const float* __restrict__ contrast,
                                                    const float* __restrict__ bright,
                                                    const double* __restrict__ affine, WarpGeom g,
                                                    int mode, float* __restrict__ gfac) {
  const int b = blockIdx.z;
  const int i = blockIdx.y, j = blockIdx.x * 256 + threadIdx.x;
  if (j >= g.S) return;
  const size_t plane = (size_t)g.S * g.S;
  const size_t o = (size_t)b * 3 * plane + (size_t)i * g.S + j;
  float adv[3], msk;
  bool rng[3];
  const po::Geo G = po::load_geo(affine + 6 * b, g.S);
  if (!warp_pixel(G, g, mp, noise_src(noise, g, b), contrast[b], g.pre ? 0.f : bright[b],
                  i, j, adv, msk, rng))
    return;   // never read by phase B
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const float out = adv[ch] * msk;
    float gv = d_out[o + ch * plane];
    if (mode == 1 && out == 0.f) gv = 0.f;
    gv = gv * msk;                                 // d(clamp(adv)*msk)/d clamp(adv)
    if (!rng[ch]) gv = 0.f;                        // clamp backward (inclusive bounds)
    gfac[o + ch * plane] = gv;
  }
}

// Phase A with four consecutive pixels of a row per thread (S % 4 == 0), as
// warp_fwd4_k: a quarter of the threads of warp_bwd_a_k over the full frame;
// a quad with a footprint pixel loads d_out and stores gfac as 16-byte
// vectors (0 at its non-footprint pixels, which phase B never reads).  The
// per-pixel arithmetic is warp_bwd_a_k's (bit-identical factors).
__global__ __launch_bounds__(256) void warp_bwd_a4_k(const float* __restrict__ d_out,
                                                     const float* __restrict__ mp,
                                                     const float* __restrict__ noise,
                                                     const float* __restrict__ contrast,
                                                     const float* __restrict__ bright,
                                                     const double* __restrict__ affine, WarpGeom g,
                                                     int mode, float* __restrict__ gfac) {
  const int b = blockIdx.y;
  const int sq = g.S >> 2;
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= g.S * sq) return;
  const int i = q / sq, j0 = (q - i * sq) * 4;
  const size_t plane = (size_t)g.S * g.S;
  const size_t o = (size_t)b * 3 * plane + (size_t)i * g.S + j0;
  const po::Geo G = po::load_geo(affine + 6 * b, g.S);
  const NoiseSrc nz = noise_src(noise, g, b);
  const float cb = contrast[b], bb = g.pre ? 0.f : bright[b];
  float adv[4][3], msk[4];
  bool rng[4][3], hit[4];
  bool any = false;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    hit[u] = warp_pixel(G, g, mp, nz, cb, bb, i, j0 + u, adv[u], msk[u], rng[u]);
    any |= hit[u];
  }
  if (!any) return;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const float4 d4 = *reinterpret_cast<const float4*>(d_out + o + ch * plane);
    const float dv[4] = {d4.x, d4.y, d4.z, d4.w};
    float gv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float out = adv[u][ch] * msk[u];
      float t = dv[u];
      if (mode == 1 && out == 0.f) t = 0.f;
      t = t * msk[u];
      if (!rng[u][ch]) t = 0.f;
      gv[u] = hit[u] ? t : 0.f;
    }
    *reinterpret_cast<float4*>(gfac + o + ch * plane) = make_float4(gv[0], gv[1], gv[2], gv[3]);
  }
}

// Backward phase B: per patch element (pr, pc), gather over images and over the
// output pixels whose bilinear footprint covers padded-input pixel (pr+padT, pc+padL).
// A workgroup holds WB_EL patch elements x WB_G image groups: group q sums the
// images q, q + WB_G, ... in increasing order, then the WB_G partials are added
// in group order through LDS (deterministic, no atomics, no workspace); the
// batch is spread over WB_G x more workgroups than one thread per element.
// Only the output pixels whose sample point lies in [c-1, c+1) x [r-1, r+1)
// can have (r, c) as a corner, so the scan covers the integer points of that
// square's preimage box (from the inverse map with one division per image;
// +-1e-6 px against its rounding) instead of the box widened by one pixel on
// each side (the round-2 scan): for a down-scaled patch (an output pixel spans
// several patch pixels) that is ~0-1 candidate pixels per (element, image)
// instead of >= 9.  The skipped pixels fail the corner test anyway, so the
// contributions and their order (rows, then columns) are unchanged.  (A fused
// single pass that recomputes phase A at each candidate instead of reading
// gfac measured 477 us against 165 + 159 us on tiny B=256: each footprint
// pixel is the candidate of 4 corners, and warp_pixel's 24 gathers dominate.)
// Per-image terms (the pixel-space map, its inverse, contrast, brightness)
// are formed once per workgroup into LDS, WB_CH images at a time, instead of
// once per (element, image) pair (the same double values, so the same bits).
// 32 image groups x 8 elements per workgroup: 4x the threads of an
// element-major split, to hide the candidates' dependent gfac loads (batches
// of more than 32 images; smaller ones keep 8 groups x 32 elements, whose
// groups all hold images).
// Per image the table holds the scan terms (the float64 map's inverse, fp32,
// with the window margins) and the sample-point terms: the fp32 theta of a
// reference-form row or the float64 pixel-space map.
//
// One candidate path serves both forms (one compiled bilinear step keeps the
// kernel at 94 VGPRs, 5 waves per SIMD; a per-form dispatch of the whole step
// measured 180 against 143 us on tiny B=256, factor pass included): the
// reference form's fp32 coordinate is widened to float64 exactly and goes
// through the float64 form's floor and weights.  That is bit-exact for every
// coordinate >= 1 -- floor is exact, e = x - floor(x) is exact in fp32 and in
// float64, 1 - e is exact in fp32 (e is a multiple of ulp(x) >= 2^-23), and a
// product of two fp32 values is exact in float64, so rounding it once to fp32
// is the fp32 product -- and phase B only meets coordinates >= pad - 1 (the
// corner it serves lies in the padded patch region), so launches with pad >= 2
// use it (EXACTD); others compute the reference form's weights in fp32.
constexpr int WB_CH = 256;     // images per LDS table chunk (WB_CH x 96 B)
struct WarpInv {
  float4 m;                    // the inverse's linear part m00, m01, m10, m11
  float4 t;                    // a02, a12, and the window half-widths hj, hi
  union {
    double af[6];              // form 0: the float64 pixel-space map
    float th[6];               // forms 1, 2: the fp32 theta
  };
  float cb, bb;
  int form;
};
// image b's scan and sample-point terms, contrast, brightness
__device__ __forceinline__ WarpInv make_inv(const double* row, int S, float cb, float bb) {
  WarpInv w;
  const po::Geo G = po::load_geo(row, S);
  const double* a = G.af;
  const double det = a[0] * a[4] - a[1] * a[3];
  const double inv = 1.0 / det;
  const float m00 = (float)(a[4] * inv), m01 = (float)(-a[1] * inv);
  const float m10 = (float)(-a[3] * inv), m11 = (float)(a[0] * inv);
  // window half-widths: the preimage of the corner square, widened by the
  // scan's own fp32 rounding (1e-3 px covers |error| < 1e-4 px at these sizes)
  // and, for the reference forms, by the distance d of the fp32 sample points
  // from the float64 map: a candidate's exact sample point lies within 1 + d of
  // (c, r), d <= (S/2) u (6 (|t0| + |t1|) + 4 |t2| + 1) + u (S + 1) (u = 2^-24:
  // the base, product, sum and fma roundings of ref_sample_coord), taken twice
  float grow = 1.0f;
  if (G.ref) {
    const double u = 0x1p-24, hS = 0.5 * S;
    double t[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) t[k] = fabs((double)G.th[k]);
    const double dx = hS * u * (6.0 * (t[0] + t[1]) + 4.0 * t[2] + 1.0) + u * (S + 1);
    const double dy = hS * u * (6.0 * (t[3] + t[4]) + 4.0 * t[5] + 1.0) + u * (S + 1);
    grow = (float)(1.0 + 2.0 * fmax(dx, dy));
  }
  w.m = make_float4(m00, m01, m10, m11);
  w.t = make_float4((float)a[2], (float)a[5], (fabsf(m00) + fabsf(m01)) * grow + 1e-3f,
                    (fabsf(m10) + fabsf(m11)) * grow + 1e-3f);
  w.form = G.ref;
  if (G.ref) {
#pragma unroll
    for (int k = 0; k < 6; ++k) w.th[k] = G.th[k];
  } else {
#pragma unroll
    for (int k = 0; k < 6; ++k) w.af[k] = G.af[k];
  }
  w.cb = cb;
  w.bb = bb;
  return w;
}

// IL: gfac interleaved [B][S][S][4] (the footprint-box forms: one 16-byte load
// per candidate pixel instead of one 4-byte load from each of three planes).
template <int WB_EL, int WB_G, bool IL, bool EXACTD>
__global__ __launch_bounds__(256) void warp_bwd_b_k(const float* __restrict__ gfac, const float* __restrict__ mp,
                                                    const float* __restrict__ noise,
                                                    const float* __restrict__ contrast,
                                                    const float* __restrict__ bright,
                                                    const double* __restrict__ affine, WarpGeom g, int B,
                                                    float* __restrict__ d_mp, int xr) {
  __shared__ float part[3][WB_G][WB_EL];
  __shared__ WarpInv tab[WB_CH];
  const int el = threadIdx.x % WB_EL, q = threadIdx.x / WB_EL;
  // xr: consecutive element blocks on one XCD (a band of patch rows per XCD):
  // neighbouring elements share candidate pixels, whose gfac lines then stay
  // in that XCD's L2 instead of being fetched by several
  const int blk = xr ? po::xcd_remap() : (int)blockIdx.x;
  const int e0 = blk * WB_EL + el;
  const bool live = e0 < g.P * g.P;
  const int e = live ? e0 : 0;
  const int pr = e / g.P, pc = e % g.P;
  const int r = pr + g.padT, c = pc + g.padL;
  const size_t plane = (size_t)g.S * g.S;
  // the element's patch values (the clamp test's t = mp * contrast + bright),
  // requested once before the table build instead of after each image's
  // candidate gathers (one dependent round trip less per image)
  float mpv[3] = {0.f, 0.f, 0.f};
  if (!g.pre)
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) mpv[ch] = mp[((size_t)ch * g.P + pr) * g.P + pc];
  float d0 = 0.f, d1 = 0.f, d2 = 0.f;
  for (int bc = 0; bc < B; bc += WB_CH) {
    const int nb = min(WB_CH, B - bc);
    // (a table phase A writes once per launch, read through the cache instead of
    // built per workgroup in LDS, measured slower: 140 -> 158 us on tiny B=256)
    if (bc) __syncthreads();                  // the previous chunk's readers are done
    for (int t = threadIdx.x; t < nb; t += 256)
      tab[t] = make_inv(affine + 6 * (bc + t), g.S, contrast[bc + t], g.pre ? 0.f : bright[bc + t]);
    __syncthreads();
    for (int bl = q; bl < (live ? nb : 0); bl += WB_G) {
      const int b = bc + bl;
      // output pixels whose sample point can have (r, c) as a bilinear corner:
      // the preimage of (c-1, c+1) x (r-1, r+1) under the pixel-space affine,
      // evaluated in fp32 with make_inv's margins: a wider scan only tests more
      // pixels, each with its exact sample point, so the candidates and their
      // order are unchanged
      const float4 m = tab[bl].m, tw = tab[bl].t;
      const float X = (float)c - tw.x, Y = (float)r - tw.y;
      const float jc = m.x * X + m.y * Y, ic = m.z * X + m.w * Y;
      const float jl = fmaxf(ceilf(jc - tw.z), 0.f), jh = fminf(floorf(jc + tw.z), (float)(g.S - 1));
      const float il = fmaxf(ceilf(ic - tw.w), 0.f), ih = fminf(floorf(ic + tw.w), (float)(g.S - 1));
      if (!(jl <= jh && il <= ih)) continue;                 // no pixel of the frame (or a NaN map)
      const int j0 = (int)jl, j1 = (int)jh, i0 = (int)il, i1 = (int)ih;
      const WarpInv& w = tab[bl];
      const int form = w.form;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f;
      bool cand = false;
      const float* gb = gfac + (size_t)b * (IL ? 4 : 3) * plane;
      for (int i = i0; i <= i1; ++i)
        for (int j = j0; j <= j1; ++j) {
          int x0, y0;
          float wb[4];
          if (EXACTD || !form) {
            double ix, iy;
            if (form) {
              float fx, fy;
              po::ref_sample_coord(w.th, form, g.ax, i, j, fx, fy);
              ix = fx;
              iy = fy;
            } else {
              sample_coord(w.af, i, j, ix, iy);
            }
            bilinear(ix, iy, x0, y0, wb);
          } else if (!sample_point_ref(w.th, form, g, i, j, x0, y0, wb)) {
            continue;
          }
          const int dx = c - x0, dy = r - y0;
          if (dx < 0 || dx > 1 || dy < 0 || dy > 1) continue;
          const float wt = wb[2 * dy + dx];
          const size_t o = (size_t)i * g.S + j;
          float gv[3];
          if constexpr (IL) {
            const float4 v4 = *reinterpret_cast<const float4*>(gb + 4 * o);
            gv[0] = v4.x;
            gv[1] = v4.y;
            gv[2] = v4.z;
          } else {
            gv[0] = gb[o];
            gv[1] = gb[o + plane];
            gv[2] = gb[o + 2 * plane];
          }
          a0 += wt * gv[0];
          a1 += wt * gv[1];
          a2 += wt * gv[2];
          cand = true;
        }
      // no output pixel of this image has (r, c) as a corner: its term is +0
      // (a = +0, contrast > 0), and adding +0 never changes d (which starts at
      // +0 and so is never -0), so the image is skipped exactly -- and with it
      // the pre-augmented value (keyed: a Philox call) the clamp test needs
      if (!cand) continue;
      const float cb = w.cb, bb = w.bb;
      const NoiseSrc nz = noise_src(noise, g, b);
      // through clamp(adv*contrast + bright + noise) and * contrast, summed over images
      const float av[3] = {a0, a1, a2};
      float dd[3];
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        const size_t po_ = ((size_t)ch * g.P + pr) * g.P + pc;
        bool in;
        if (nz.pre) {
          const float pre = nz.pre[po_];
          in = pre >= 0.f && pre <= 1.f;
        } else {
          // pre = fl(t + fl(0.1 nz)), t = fl(fl(mp cb) + bb), |fl(0.1 nz)| <= 0.1f
          // (nz in [-1, 1)): rounding is monotonic, so pre lies in [fl(t - 0.1f),
          // fl(t + 0.1f)], and when that interval is inside [0, 1] the clamp
          // test passes whatever the noise -- its Philox call is skipped
          const float t = mpv[ch] * cb + bb;
          if (t - 0.1f >= 0.f && t + 0.1f <= 1.f) {
            in = true;
          } else {
            const float pre = t + nz.at(po_) * 0.1f;
            in = pre >= 0.f && pre <= 1.f;
          }
        }
        dd[ch] = in ? av[ch] * cb : 0.f;
      }
      d0 += dd[0]; d1 += dd[1]; d2 += dd[2];
    }
  }
  __syncthreads();
  part[0][q][el] = d0;
  part[1][q][el] = d1;
  part[2][q][el] = d2;
  __syncthreads();
  if (q < 3 && live) {
    float t = part[q][0][el];
#pragma unroll
    for (int k = 1; k < WB_G; ++k) t += part[q][k][el];
    d_mp[e + (size_t)q * g.P * g.P] = t;
  }
}

template <bool EXACTD>
void launch_bwd_b_x(const float* gfac, const float* mp, const float* noise, const float* contrast,
                    const float* bright, const double* affine, const WarpGeom& g, int B, int P, float* d_mp,
                    hipStream_t st, bool il, int xr) {
  if (B > 32) {
    if (il)
      hipLaunchKernelGGL((warp_bwd_b_k<8, 32, true, EXACTD>), dim3(po::ceil_div(P * P, 8)), dim3(256), 0, st, gfac,
                         mp, noise, contrast, bright, affine, g, B, d_mp, xr);
    else
      hipLaunchKernelGGL((warp_bwd_b_k<8, 32, false, EXACTD>), dim3(po::ceil_div(P * P, 8)), dim3(256), 0, st, gfac,
                         mp, noise, contrast, bright, affine, g, B, d_mp, xr);
  } else {
    if (il)
      hipLaunchKernelGGL((warp_bwd_b_k<32, 8, true, EXACTD>), dim3(po::ceil_div(P * P, 32)), dim3(256), 0, st, gfac,
                         mp, noise, contrast, bright, affine, g, B, d_mp, xr);
    else
      hipLaunchKernelGGL((warp_bwd_b_k<32, 8, false, EXACTD>), dim3(po::ceil_div(P * P, 32)), dim3(256), 0, st,
                         gfac, mp, noise, contrast, bright, affine, g, B, d_mp, xr);
  }
}

void launch_bwd_b(const float* gfac, const float* mp, const float* noise, const float* contrast, const float* bright,
                  const double* affine, const WarpGeom& g, int B, int P, float* d_mp, hipStream_t st,
                  bool il = false) {
  static const int xr = [] {
    const char* e = getenv("ADVPATCH_WARP_XCD");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  if (g.padL >= 2 && g.padT >= 2)
    launch_bwd_b_x<true>(gfac, mp, noise, contrast, bright, affine, g, B, P, d_mp, st, il, xr);
  else
    launch_bwd_b_x<false>(gfac, mp, noise, contrast, bright, affine, g, B, P, d_mp, st, il, xr);
}

// L patches per image composited in slot order (PatchApplier, load_data.py:
// 808-833, over the [B,L,3,S,S] output of PatchTransformer_vanishing): per
// element the value of the last slot whose clamp(adv)*msk is non-zero, else
// the image.  Slots are visited last to first and a pixel outside a slot's
// footprint box skips it; the per-slot value is warp_pixel's, so the result
// equals L sequential po_warp_fwd + po_apply_fwd passes bit for bit.
template <bool AUG>
__global__ __launch_bounds__(256) void warp_multi_k(const float* __restrict__ img, const float* __restrict__ mp,
                                                    const float* __restrict__ noise,
                                                    const float* __restrict__ contrast,
                                                    const float* __restrict__ bright,
                                                    const double* __restrict__ affine,
                                                    const int32_t* __restrict__ roi, int L, WarpGeom g,
                                                    float* __restrict__ out) {
  const int b = blockIdx.y;
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= g.S * g.S) return;
  const int i = q / g.S, j = q - i * g.S;
  const size_t plane = (size_t)g.S * g.S;
  const size_t o = (size_t)b * 3 * plane + q;
  float v[3] = {0.f, 0.f, 0.f};
  bool set[3] = {false, false, false};
  for (int l = L - 1; l >= 0; --l) {
    const int t = b * L + l;
    const int32_t* r = roi + 4 * t;
    if (j < r[0] || j >= r[2] || i < r[1] || i >= r[3]) continue;
    float adv[3], msk;
    bool rng[3];
    const NoiseSrc nz = noise_src(AUG ? noise : nullptr, g, t);     // !AUG: never read
    const po::Geo G = po::load_geo(affine + 6 * t, g.S);
    if (!warp_pixel<AUG>(G, g, mp, nz, AUG ? contrast[t] : 1.f, AUG ? bright[t] : 0.f, i, j, adv,
                         msk, rng))
      continue;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const float val = adv[ch] * msk;                  // load_data.py:1227-1230
      if (!set[ch] && val != 0.f) { v[ch] = val; set[ch] = true; }
    }
    if (set[0] && set[1] && set[2]) break;
  }
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) out[o + ch * plane] = set[ch] ? v[ch] : img[o + ch * plane];
}

WarpGeom make_geom(int S, int P, uint64_t seed = 0, uint64_t counter = 0, int b0 = 0) {
  WarpGeom g;
  g.S = S;
  g.P = P;
  g.nk0 = (uint32_t)seed;
  g.nk1 = (uint32_t)(seed >> 32);
  g.nc_lo = (uint32_t)counter;
  g.nc_hi = (uint32_t)(counter >> 32);
  g.nb0 = b0;
  g.pre = nullptr;
  const double pad = (S - P) / 2.0;      // load_data.py:534
  g.padL = (int)(pad + 0.5);            // ConstantPad2d((int(pad+.5), int(pad), int(pad+.5), int(pad)))
  g.padT = (int)(pad + 0.5);
  g.ax = po::ref_axis(S);
  return g;
}
}  // namespace

namespace {
int warp_fwd(const float* img, const float* patch_mp, const float* noise, const float* contrast, const float* bright,
             const double* affine, int B, int S, int mode, float* out, const WarpGeom& g, po_stream_t s) {
  if (S % 4 == 0 && ((uintptr_t)img | (uintptr_t)out) % 16 == 0) {
    hipLaunchKernelGGL(warp_fwd4_k, dim3(po::ceil_div(S * (S / 4), 256), B), dim3(256), 0, po::stream_of(s), img,
                       patch_mp, noise, contrast, bright, affine, g, mode, out);
    return po::check_launch("po_warp_fwd");
  }
  dim3 grid(po::ceil_div(S, 256), S, B);
  hipLaunchKernelGGL(warp_fwd_k, grid, dim3(256), 0, po::stream_of(s), img, patch_mp, noise, contrast,
                     bright, affine, g, mode, out);
  return po::check_launch("po_warp_fwd");
}
}  // namespace

extern "C" int po_warp_fwd(const float* img, const float* patch_mp, const float* noise,
                           const float* contrast, const float* bright, const double* affine, int B,
                           int S, int P, int mode, float* out, po_stream_t s) {
  PO_REQUIRE(patch_mp && noise && contrast && bright && affine && out, "po_warp_fwd: null pointer");
  PO_REQUIRE(mode == 0 || (mode == 1 && img), "po_warp_fwd: mode must be 0 or 1 (1 needs img)");
  PO_REQUIRE(B > 0 && S > 1 && P > 0 && P <= S, "po_warp_fwd: bad shape B=%d S=%d P=%d", B, S, P);
  return warp_fwd(img, patch_mp, noise, contrast, bright, affine, B, S, mode, out, make_geom(S, P), s);
}

extern "C" int po_warp_fwd_keyed(const float* img, const float* patch_mp, uint64_t seed, uint64_t counter, int b0,
                                 const float* contrast, const float* bright, const double* affine, int B, int S, int P,
                                 int mode, float* out, po_stream_t s) {
  PO_REQUIRE(patch_mp && contrast && bright && affine && out, "po_warp_fwd_keyed: null pointer");
  PO_REQUIRE(mode == 0 || (mode == 1 && img), "po_warp_fwd_keyed: mode must be 0 or 1 (1 needs img)");
  PO_REQUIRE(B > 0 && S > 1 && P > 0 && P <= S && b0 >= 0, "po_warp_fwd_keyed: bad shape B=%d S=%d P=%d", B, S, P);
  PO_REQUIRE(3LL * P * P < (1LL << 31), "po_warp_fwd_keyed: patch too large");
  return warp_fwd(img, patch_mp, nullptr, contrast, bright, affine, B, S, mode, out, make_geom(S, P, seed, counter, b0),
                  s);
}

namespace {
int warp_bwd(const float* d_out, const float* patch_mp, const float* noise, const float* contrast, const float* bright,
             const double* affine, int B, int S, int P, int mode, float* work, float* d_patch_mp, const WarpGeom& g,
             po_stream_t s) {
  const bool quad = S % 4 == 0 && ((uintptr_t)d_out | (uintptr_t)work) % 16 == 0 && work != d_out;
  if (quad) {
    hipLaunchKernelGGL(warp_bwd_a4_k, dim3(po::ceil_div(S * (S / 4), 256), B), dim3(256), 0, po::stream_of(s), d_out,
                       patch_mp, noise, contrast, bright, affine, g, mode, work);
  } else {
    dim3 grid(po::ceil_div(S, 256), S, B);
    hipLaunchKernelGGL(warp_bwd_a_k, grid, dim3(256), 0, po::stream_of(s), d_out, patch_mp, noise,
                       contrast, bright, affine, g, mode, work);
  }
  int rc = po::check_launch("po_warp_bwd(a)");
  if (rc) return rc;
  launch_bwd_b(work, patch_mp, noise, contrast, bright, affine, g, B, P, d_patch_mp, po::stream_of(s));
  return po::check_launch("po_warp_bwd(b)");
}
}  // namespace

extern "C" int po_warp_bwd(const float* d_out, const float* patch_mp, const float* noise,
                           const float* contrast, const float* bright, const double* affine, int B,
                           int S, int P, int mode, float* work, float* d_patch_mp, po_stream_t s) {
  PO_REQUIRE(d_out && patch_mp && noise && contrast && bright && affine && work && d_patch_mp,
             "po_warp_bwd: null pointer");
  PO_REQUIRE(mode == 0 || mode == 1, "po_warp_bwd: mode must be 0 or 1");
  PO_REQUIRE(B > 0 && S > 1 && P > 0 && P <= S, "po_warp_bwd: bad shape");
  return warp_bwd(d_out, patch_mp, noise, contrast, bright, affine, B, S, P, mode, work, d_patch_mp, make_geom(S, P),
                  s);
}

extern "C" int po_warp_bwd_keyed(const float* d_out, const float* patch_mp, uint64_t seed, uint64_t counter, int b0,
                                 const float* contrast, const float* bright, const double* affine, int B, int S, int P,
                                 int mode, float* work, float* d_patch_mp, po_stream_t s) {
  PO_REQUIRE(d_out && patch_mp && contrast && bright && affine && work && d_patch_mp,
             "po_warp_bwd_keyed: null pointer");
  PO_REQUIRE(mode == 0 || mode == 1, "po_warp_bwd_keyed: mode must be 0 or 1");
  PO_REQUIRE(B > 0 && S > 1 && P > 0 && P <= S && b0 >= 0, "po_warp_bwd_keyed: bad shape");
  PO_REQUIRE(3LL * P * P < (1LL << 31), "po_warp_bwd_keyed: patch too large");
  return warp_bwd(d_out, patch_mp, nullptr, contrast, bright, affine, B, S, P, mode, work, d_patch_mp,
                  make_geom(S, P, seed, counter, b0), s);
}

namespace {
// The transformer's augmentation of the median-pooled patch for each image,
// before the clamp (load_data.py:548-571): pre[b][e] = mp[e] * contrast[b] +
// bright[b] + 0.1 * noise(b, e), the noise regenerated from the po_draws key
// (philox_noise's values: one Philox call per group of 4 elements, so a
// thread forms 4 consecutive elements).  The warp kernels then gather these
// values (po_warp_*_pre) instead of forming them at every bilinear corner:
// one Philox call per 4 patch elements instead of one per corner read.
__global__ __launch_bounds__(256) void augment_k(const float* __restrict__ mp, const float* __restrict__ contrast,
                                                 const float* __restrict__ bright, WarpGeom g, int n,
                                                 float* __restrict__ pre) {
  const int b = blockIdx.y;
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int e0 = 4 * t;
  if (e0 >= n) return;
  const po::u4 r = po::philox4x32_10(po::u4{(uint32_t)t, (uint32_t)(g.nb0 + b), g.nc_lo, g.nc_hi}, g.nk0, g.nk1);
  const uint32_t x[4] = {r.x, r.y, r.z, r.w};
  const float cb = contrast[b], bb = bright[b];
  float* o = pre + (size_t)b * n;
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    const int e = e0 + l;
    if (e < n) {
      const float nz = po::philox_affine(po::philox_unif(x[l]), 2.0f, -1.0f);
      o[e] = mp[e] * cb + bb + nz * 0.1f;
    }
  }
}

// ---- footprint-box form of the warp (po_warp_*_pre with the footprint boxes
// po_patch_params writes, roi [B][4] = {x0, y0, x1, y1}: no output pixel outside
// its image's box samples the padded patch region).  The box is widened to whole
// pixel quads [qx0, qx1) (qx0 = x0 & ~3): warp_quad_copy_k writes the quads
// outside it (the image in mode 1, zeros in mode 0) as 16-byte copies with no
// per-pixel geometry, warp_box_fwd_k / warp_box_bwd_a_k run warp_pixel over the
// box's pixels, one per thread (the footprint is a few percent of the frame:
// spread over many waves instead of a few heavy quads).  Same per-pixel
// arithmetic as warp_fwd4_k / warp_bwd_a4_k, so bit-identical outputs.
using po::QBox;
using po::quad_box;

__global__ __launch_bounds__(256) void warp_quad_copy_k(const float* __restrict__ img, const int32_t* __restrict__ roi,
                                                        int S, int mode, float* __restrict__ out) {
  const int b = blockIdx.y;
  const int sq = S >> 2;
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= S * sq) return;
  const int i = q / sq, j0 = (q - i * sq) * 4;
  const QBox bx = quad_box(roi, b, S);
  if (i >= bx.y0 && i < bx.y1 && j0 >= bx.qx0 && j0 < bx.qx1) return;    // warp_box_fwd_k's quad
  const size_t plane = (size_t)S * S;
  const size_t o = (size_t)b * 3 * plane + (size_t)i * S + j0;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const float4 v = mode == 1 ? *reinterpret_cast<const float4*>(img + o + ch * plane) : make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(out + o + ch * plane) = v;
  }
}

// one box pixel of the forward
__device__ __forceinline__ void box_fwd_pixel(const float* __restrict__ img, const float* __restrict__ mp,
                                              const po::Geo& G, const NoiseSrc& nz, float cb, float bb,
                                              const WarpGeom& g, int mode, int b, int i, int j,
                                              float* __restrict__ out, float* __restrict__ fac) {
  const size_t plane = (size_t)g.S * g.S;
  const size_t o = (size_t)b * 3 * plane + (size_t)i * g.S + j;
  float adv[3], msk;
  bool rng[3];
  const bool hit = warp_pixel(G, g, mp, nz, cb, bb, i, j, adv, msk, rng);
  float f4[4] = {-1.f, -1.f, -1.f, -1.f};
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    float v = hit ? adv[ch] * msk : 0.f;                       // load_data.py:791-792
    // the backward's factor: d_out * msk where the gradient passes (clamp in
    // range, and in mode 1 the patch value not replaced by the frame), else
    // the sentinel -1 for an exact +0 (warp_box_bwd_a_k's rule)
    if (hit && rng[ch] && !(mode == 1 && v == 0.f)) f4[ch] = msk;
    if (mode == 1) v = (v == 0.f) ? img[o + ch * plane] : v;   // load_data.py:820
    out[o + ch * plane] = v;
  }
  if (fac)
    *reinterpret_cast<float4*>(fac + ((size_t)b * plane + (size_t)i * g.S + j) * 4) =
        make_float4(f4[0], f4[1], f4[2], f4[3]);
}

__global__ __launch_bounds__(256) void warp_box_fwd_k(const float* __restrict__ img, const float* __restrict__ mp,
                                                      const float* __restrict__ contrast,
                                                      const float* __restrict__ bright,
                                                      const double* __restrict__ affine,
                                                      const int32_t* __restrict__ roi, WarpGeom g, int mode,
                                                      float* __restrict__ out, float* __restrict__ fac) {
  const int b = blockIdx.y;
  const QBox bx = quad_box(roi, b, g.S);
  const int bw = bx.qx1 - bx.qx0, area = bw * (bx.y1 - bx.y0);
  const NoiseSrc nz = noise_src(nullptr, g, b);
  // pre-augmented values (g.pre) or mp + the draws + the keyed noise at each corner
  const float cb = g.pre ? 1.f : contrast[b], bb = g.pre ? 0.f : bright[b];
  const po::Geo G = po::load_geo(affine + 6 * b, g.S);
  if (blockIdx.x * 256 >= area) return;                        // (uniform) no pixel of the box here
  for (int p = blockIdx.x * 256 + threadIdx.x; p < area; p += gridDim.x * 256) {
    const int r = p / bw;
    box_fwd_pixel(img, mp, G, nz, cb, bb, g, mode, b, bx.y0 + r, bx.qx0 + (p - r * bw), out, fac);
  }
}

// phase A of the backward over the footprint box only (phase B reads gfac at
// footprint pixels only), gfac interleaved [B][S][S][4]: one 16-byte store
// per pixel, read back by phase B as one 16-byte load per candidate
__global__ __launch_bounds__(256) void warp_box_bwd_a_k(const float* __restrict__ d_out,
                                                        const float* __restrict__ mp,
                                                        const float* __restrict__ contrast,
                                                        const float* __restrict__ bright,
                                                        const double* __restrict__ affine,
                                                        const int32_t* __restrict__ roi, WarpGeom g, int mode,
                                                        float* __restrict__ gfac) {
  const int b = blockIdx.y;
  const QBox bx = quad_box(roi, b, g.S);
  const int bw = bx.qx1 - bx.qx0, area = bw * (bx.y1 - bx.y0);
  const size_t plane = (size_t)g.S * g.S;
  const NoiseSrc nz = noise_src(nullptr, g, b);
  const float cb = contrast[b], bb = g.pre ? 0.f : bright[b];
  const po::Geo G = po::load_geo(affine + 6 * b, g.S);
  if (blockIdx.x * 256 >= area) return;                        // (uniform) no pixel of the box here
  for (int p = blockIdx.x * 256 + threadIdx.x; p < area; p += gridDim.x * 256) {
    const int r = p / bw;
    const int i = bx.y0 + r, j = bx.qx0 + (p - r * bw);
    const size_t o = (size_t)b * 3 * plane + (size_t)i * g.S + j;
    float adv[3], msk;
    bool rng[3];
    if (!warp_pixel(G, g, mp, nz, cb, bb, i, j, adv, msk, rng)) continue;
    float gv4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const float outv = adv[ch] * msk;
      float gv = d_out[o + ch * plane];
      if (mode == 1 && outv == 0.f) gv = 0.f;
      gv = gv * msk;
      if (!rng[ch]) gv = 0.f;
      gv4[ch] = gv;
    }
    *reinterpret_cast<float4*>(gfac + ((size_t)b * plane + (size_t)i * g.S + j) * 4) =
        make_float4(gv4[0], gv4[1], gv4[2], gv4[3]);
  }
}

// phase A from the forward's factors (po_warp_box_fwd_fac): no warp_pixel
// recomputation -- a 16-byte factor load, the three d_out loads and the gfac
// store in place of the factors.  The same products as warp_box_bwd_a_k
// (d_out * msk where the gradient passes, +0 elsewhere), so the same bits.
__device__ __forceinline__ void box_fac_pixel(const float* __restrict__ d_out, int S, int b, int i, int j,
                                              float* __restrict__ fac) {
  const size_t plane = (size_t)S * S;
  const size_t o = (size_t)b * 3 * plane + (size_t)i * S + j;
  float4* fp = reinterpret_cast<float4*>(fac + ((size_t)b * plane + (size_t)i * S + j) * 4);
  const float4 f = *fp;
  const float fv[3] = {f.x, f.y, f.z};
  float gv[3];
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) gv[ch] = fv[ch] < 0.f ? 0.f : d_out[o + ch * plane] * fv[ch];
  *fp = make_float4(gv[0], gv[1], gv[2], 0.f);
}

__global__ __launch_bounds__(256) void warp_box_bwd_fac_k(const float* __restrict__ d_out,
                                                          const int32_t* __restrict__ roi, int S,
                                                          float* __restrict__ fac) {
  const int b = blockIdx.y;
  const QBox bx = quad_box(roi, b, S);
  const int bw = bx.qx1 - bx.qx0, area = bw * (bx.y1 - bx.y0);
  for (int p = blockIdx.x * 256 + threadIdx.x; p < area; p += gridDim.x * 256) {
    const int r = p / bw;
    box_fac_pixel(d_out, S, b, bx.y0 + r, bx.qx0 + (p - r * bw), fac);
  }
}

// workgroups per image of the box kernels: enough for a box of an eighth of the
// frame in one pass (a larger box loops)
__host__ inline int box_blocks(int S) { return po::ceil_div(po::ceil_div((int64_t)S * S, 8), 256); }
}  // namespace

extern "C" int po_augment_patch(const float* patch_mp, uint64_t seed, uint64_t counter, int b0, const float* contrast,
                                const float* bright, int B, int P, float* pre, po_stream_t s) {
  PO_REQUIRE(patch_mp && contrast && bright && pre, "po_augment_patch: null pointer");
  PO_REQUIRE(B > 0 && P > 0 && b0 >= 0 && 3LL * P * P < (1LL << 31), "po_augment_patch: bad shape B=%d P=%d", B, P);
  const int n = 3 * P * P;
  WarpGeom g = make_geom(P, P, seed, counter, b0);
  hipLaunchKernelGGL(augment_k, dim3(po::ceil_div(po::ceil_div(n, 4), 256), B), dim3(256), 0, po::stream_of(s),
                     patch_mp, contrast, bright, g, n, pre);
  return po::check_launch("po_augment_patch");
}

extern "C" int po_warp_fwd_pre(const float* img, const float* pre, const double* affine, const int32_t* roi, int B,
                               int S, int P, int mode, float* out, po_stream_t s) {
  PO_REQUIRE(pre && affine && roi && out, "po_warp_fwd_pre: null pointer");
  PO_REQUIRE(mode == 0 || (mode == 1 && img), "po_warp_fwd_pre: mode must be 0 or 1 (1 needs img)");
  PO_REQUIRE(B > 0 && S > 1 && P > 0 && P <= S, "po_warp_fwd_pre: bad shape B=%d S=%d P=%d", B, S, P);
  PO_REQUIRE(3LL * P * P < (1LL << 31) && (int64_t)B * 3 * S * S < (1LL << 40), "po_warp_fwd_pre: too large");
  WarpGeom g = make_geom(S, P);
  g.pre = pre;
  if (S % 4 != 0 || ((uintptr_t)img | (uintptr_t)out) % 16 != 0)      // whole-frame one-pixel kernel
    return warp_fwd(img, pre, nullptr, nullptr, nullptr, affine, B, S, mode, out, g, s);
  hipStream_t st = po::stream_of(s);
  hipLaunchKernelGGL(warp_quad_copy_k, dim3(po::ceil_div(S * (S / 4), 256), B), dim3(256), 0, st, img, roi, S, mode,
                     out);
  hipLaunchKernelGGL(warp_box_fwd_k, dim3(box_blocks(S), B), dim3(256), 0, st, img, nullptr, nullptr, nullptr, affine,
                     roi, g, mode, out, nullptr);
  return po::check_launch("po_warp_fwd_pre");
}

static int box_fwd_keyed(const float* img, const float* patch_mp, uint64_t seed, uint64_t counter, int b0,
                         const float* contrast, const float* bright, const double* affine, const int32_t* roi, int B,
                         int S, int P, int mode, int fill, float* out, float* fac, po_stream_t s) {
  PO_REQUIRE(patch_mp && contrast && bright && affine && roi && out, "po_warp_box_fwd_keyed: null pointer");
  PO_REQUIRE(mode == 0 || (mode == 1 && img), "po_warp_box_fwd_keyed: mode must be 0 or 1 (1 needs img)");
  PO_REQUIRE(B > 0 && S > 1 && P > 0 && P <= S && b0 >= 0 && S % 4 == 0,
             "po_warp_box_fwd_keyed: bad shape B=%d S=%d P=%d (S %% 4 == 0)", B, S, P);
  PO_REQUIRE(3LL * P * P < (1LL << 31) && (int64_t)B * 3 * S * S < (1LL << 40), "po_warp_box_fwd_keyed: too large");
  PO_REQUIRE(!fill || ((uintptr_t)img | (uintptr_t)out) % 16 == 0, "po_warp_box_fwd_keyed: fill needs 16-byte alignment");
  const WarpGeom g = make_geom(S, P, seed, counter, b0);
  hipStream_t st = po::stream_of(s);
  if (fill)
    hipLaunchKernelGGL(warp_quad_copy_k, dim3(po::ceil_div(S * (S / 4), 256), B), dim3(256), 0, st, img, roi, S, mode,
                       out);
  hipLaunchKernelGGL(warp_box_fwd_k, dim3(box_blocks(S), B), dim3(256), 0, st, img, patch_mp, contrast, bright, affine,
                     roi, g, mode, out, fac);
  return po::check_launch("po_warp_box_fwd_keyed");
}

extern "C" int po_warp_box_fwd_keyed(const float* img, const float* patch_mp, uint64_t seed, uint64_t counter, int b0,
                                     const float* contrast, const float* bright, const double* affine,
                                     const int32_t* roi, int B, int S, int P, int mode, int fill, float* out,
                                     po_stream_t s) {
  return box_fwd_keyed(img, patch_mp, seed, counter, b0, contrast, bright, affine, roi, B, S, P, mode, fill, out,
                       nullptr, s);
}

extern "C" int po_warp_box_fwd_fac(const float* img, const float* patch_mp, uint64_t seed, uint64_t counter, int b0,
                                   const float* contrast, const float* bright, const double* affine,
                                   const int32_t* roi, int B, int S, int P, int mode, int fill, float* out, float* fac,
                                   po_stream_t s) {
  PO_REQUIRE(fac && (uintptr_t)fac % 16 == 0, "po_warp_box_fwd_fac: fac must be non-null and 16-byte aligned");
  return box_fwd_keyed(img, patch_mp, seed, counter, b0, contrast, bright, affine, roi, B, S, P, mode, fill, out, fac,
                       s);
}

extern "C" int po_warp_bwd_pre(const float* d_out, const float* pre, const float* contrast, const double* affine,
                               const int32_t* roi, int B, int S, int P, int mode, float* work, float* d_patch_mp,
                               po_stream_t s) {
  PO_REQUIRE(d_out && pre && contrast && affine && roi && work && d_patch_mp, "po_warp_bwd_pre: null pointer");
  PO_REQUIRE(mode == 0 || mode == 1, "po_warp_bwd_pre: mode must be 0 or 1");
  PO_REQUIRE(B > 0 && S > 1 && P > 0 && P <= S, "po_warp_bwd_pre: bad shape");
  PO_REQUIRE(3LL * P * P < (1LL << 31), "po_warp_bwd_pre: patch too large");
  PO_REQUIRE(work != d_out, "po_warp_bwd_pre: work may not alias d_out");
  PO_REQUIRE((uintptr_t)work % 16 == 0, "po_warp_bwd_pre: work must be 16-byte aligned");
  WarpGeom g = make_geom(S, P);
  g.pre = pre;
  hipStream_t st = po::stream_of(s);
  hipLaunchKernelGGL(warp_box_bwd_a_k, dim3(box_blocks(S), B), dim3(256), 0, st, d_out, nullptr, contrast, nullptr,
                     affine, roi, g, mode, work);
  int rc = po::check_launch("po_warp_bwd_pre(a)");
  if (rc) return rc;
  launch_bwd_b(work, pre, nullptr, contrast, nullptr, affine, g, B, P, d_patch_mp, st, true);
  return po::check_launch("po_warp_bwd_pre(b)");
}

extern "C" int po_warp_box_bwd_keyed(const float* d_out, const float* patch_mp, uint64_t seed, uint64_t counter, int b0,
                                     const float* contrast, const float* bright, const double* affine,
                                     const int32_t* roi, int B, int S, int P, int mode, float* work, float* d_patch_mp,
                                     po_stream_t s) {
  PO_REQUIRE(d_out && patch_mp && contrast && bright && affine && roi && work && d_patch_mp,
             "po_warp_box_bwd_keyed: null pointer");
  PO_REQUIRE(mode == 0 || mode == 1, "po_warp_box_bwd_keyed: mode must be 0 or 1");
  PO_REQUIRE(B > 0 && S > 1 && P > 0 && P <= S && b0 >= 0, "po_warp_box_bwd_keyed: bad shape");
  PO_REQUIRE(3LL * P * P < (1LL << 31), "po_warp_box_bwd_keyed: patch too large");
  PO_REQUIRE(work != d_out, "po_warp_box_bwd_keyed: work may not alias d_out");
  PO_REQUIRE((uintptr_t)work % 16 == 0, "po_warp_box_bwd_keyed: work must be 16-byte aligned");
  const WarpGeom g = make_geom(S, P, seed, counter, b0);
  hipStream_t st = po::stream_of(s);
  hipLaunchKernelGGL(warp_box_bwd_a_k, dim3(box_blocks(S), B), dim3(256), 0, st, d_out, patch_mp, contrast, bright,
                     affine, roi, g, mode, work);
  int rc = po::check_launch("po_warp_box_bwd_keyed(a)");
  if (rc) return rc;
  launch_bwd_b(work, patch_mp, nullptr, contrast, bright, affine, g, B, P, d_patch_mp, st, true);
  return po::check_launch("po_warp_box_bwd_keyed(b)");
}

extern "C" int po_warp_box_bwd_fac(const float* d_out, const float* patch_mp, uint64_t seed, uint64_t counter, int b0,
                                   const float* contrast, const float* bright, const double* affine,
                                   const int32_t* roi, int B, int S, int P, float* fac, float* d_patch_mp,
                                   po_stream_t s) {
  PO_REQUIRE(d_out && patch_mp && contrast && bright && affine && roi && fac && d_patch_mp,
             "po_warp_box_bwd_fac: null pointer");
  PO_REQUIRE(B > 0 && S > 1 && P > 0 && P <= S && b0 >= 0, "po_warp_box_bwd_fac: bad shape");
  PO_REQUIRE(3LL * P * P < (1LL << 31), "po_warp_box_bwd_fac: patch too large");
  PO_REQUIRE(fac != d_out, "po_warp_box_bwd_fac: fac may not alias d_out");
  PO_REQUIRE((uintptr_t)fac % 16 == 0, "po_warp_box_bwd_fac: fac must be 16-byte aligned");
  const WarpGeom g = make_geom(S, P, seed, counter, b0);
  hipStream_t st = po::stream_of(s);
  hipLaunchKernelGGL(warp_box_bwd_fac_k, dim3(box_blocks(S), B), dim3(256), 0, st, d_out, roi, S, fac);
  int rc = po::check_launch("po_warp_box_bwd_fac(a)");
  if (rc) return rc;
  launch_bwd_b(fac, patch_mp, nullptr, contrast, bright, affine, g, B, P, d_patch_mp, st, true);
  return po::check_launch("po_warp_box_bwd_fac(b)");
}

extern "C" int po_warp_composite_multi(const float* img, const float* patch_mp, const float* noise,
                                       const float* contrast, const float* bright, const double* affine,
                                       const int32_t* roi, int B, int L, int S, int P, float* out, po_stream_t s) {
  PO_REQUIRE(img && patch_mp && affine && roi && out, "po_warp_composite_multi: null pointer");
  PO_REQUIRE(!noise || (contrast && bright), "po_warp_composite_multi: noise needs contrast and bright");
  PO_REQUIRE(B > 0 && L > 0 && S > 1 && P > 0 && P <= S, "po_warp_composite_multi: bad shape B=%d L=%d S=%d P=%d",
             B, L, S, P);
  dim3 grid(po::ceil_div((int64_t)S * S, 256), B);
  if (noise)
    hipLaunchKernelGGL(warp_multi_k<true>, grid, dim3(256), 0, po::stream_of(s), img, patch_mp, noise, contrast,
                       bright, affine, roi, L, make_geom(S, P), out);
  else
    hipLaunchKernelGGL(warp_multi_k<false>, grid, dim3(256), 0, po::stream_of(s), img, patch_mp, noise, contrast,
                       bright, affine, roi, L, make_geom(S, P), out);
  return po::check_launch("po_warp_composite_multi");
}

// ------------------------------------------------------------------------
// PatchApplier on an explicit adv tensor (load_data.py:808-833)
// ------------------------------------------------------------------------
namespace {
__global__ void apply_fwd_k(const float* __restrict__ img, const float* __restrict__ adv, int64_t n,
                            float* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    float a = adv[i];
    out[i] = (a == 0.f) ? img[i] : a;
  }
}
__global__ void apply_bwd_k(const float* __restrict__ dout, const float* __restrict__ adv, int64_t n,
                            float* __restrict__ dimg, float* __restrict__ dadv) {
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    float a = adv[i], g = dout[i];
    if (dimg) dimg[i] = (a == 0.f) ? g : 0.f;
    if (dadv) dadv[i] = (a == 0.f) ? 0.f : g;
  }
}
}  // namespace

extern "C" int po_apply_fwd(const float* img, const float* adv, int64_t n, float* out, po_stream_t s) {
  PO_REQUIRE(img && adv && out && n >= 0, "po_apply_fwd: bad argument");
  if (n == 0) return PO_OK;
  hipLaunchKernelGGL(apply_fwd_k, dim3(po::ceil_div(n, 256)), dim3(256), 0, po::stream_of(s), img, adv,
                     n, out);
  return po::check_launch("po_apply_fwd");
}

extern "C" int po_apply_bwd(const float* d_out, const float* adv, int64_t n, float* d_img, float* d_adv,
                            po_stream_t s) {
  PO_REQUIRE(d_out && adv && n >= 0, "po_apply_bwd: bad argument");
  if (n == 0 || (!d_img && !d_adv)) return PO_OK;
  hipLaunchKernelGGL(apply_bwd_k, dim3(po::ceil_div(n, 256)), dim3(256), 0, po::stream_of(s), d_out,
                     adv, n, d_img, d_adv);
  return po::check_launch("po_apply_bwd");
}

// ------------------------------------------------------------------------
// Regularisers: NPS (load_data.py:357-367), TV (404-411), colour (1729-1754)
// ------------------------------------------------------------------------
namespace {
constexpr int RB = 256;        // threads per block
constexpr int RMAXB = 1024;    // max partial blocks
constexpr int NPART = 7;       // nps, tv1, tv2, s_rg, s_yb, s_rg2, s_yb2

__device__ __forceinline__ void nps_pixel(const float* col, int ncol, float r, float g, float b,
                                          float& dmin, int& kmin) {
  dmin = 0.f;
  kmin = -1;
  for (int k = 0; k < ncol; ++k) {
    float d0 = r - col[3 * k + 0] + 0.000001f;
    float d1 = g - col[3 * k + 1] + 0.000001f;
    float d2 = b - col[3 * k + 2] + 0.000001f;
    float d = sqrtf(d0 * d0 + d1 * d1 + d2 * d2 + 0.000001f);
    if (kmin < 0 || d < dmin) { dmin = d; kmin = k; }
  }
}

__device__ __forceinline__ double block_sum(double v, double* sh) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int k = 0; k < RB / 64; ++k) t += sh[k];
  return t;   // valid in thread 0
}

__global__ __launch_bounds__(RB) void reg_partial_k(const float* __restrict__ p, int P,
                                                    const float* __restrict__ col, int ncol,
                                                    double* __restrict__ part) {
  __shared__ double sh[RB / 64];
  const int n = P * P;
  double acc[NPART] = {0, 0, 0, 0, 0, 0, 0};
  const size_t pp = (size_t)n;
  for (int e = blockIdx.x * RB + threadIdx.x; e < n; e += gridDim.x * RB) {
    const int i = e / P, q = e % P;
    const float r = p[e], g = p[e + pp], b = p[e + 2 * pp];
    float dmin;
    int kmin;
    nps_pixel(col, ncol, r, g, b, dmin, kmin);
    acc[0] += dmin;
    for (int ch = 0; ch < 3; ++ch) {
      const float* pc = p + ch * pp;
      if (q + 1 < P) acc[1] += fabsf(pc[e + 1] - pc[e] + 0.000001f);
      if (i + 1 < P) acc[2] += fabsf(pc[e + P] - pc[e] + 0.000001f);
    }
    const float rg = r - g, yb = 0.5f * (r + g) - b;
    acc[3] += rg;
    acc[4] += yb;
    acc[5] += (double)rg * rg;
    acc[6] += (double)yb * yb;
  }
  for (int k = 0; k < NPART; ++k) {
    double t = block_sum(acc[k], sh);
    if (threadIdx.x == 0) part[(size_t)k * RMAXB + blockIdx.x] = t;
  }
}

// coef layout: [0]=g_nps/numel [1]=g_tv/numel [2]=g_col [3]=mu_rg [4]=mu_yb
// [5]=d sigma/d x factor [6]=d mu term / d rg_i [7]=d mu term / d yb_i
__global__ __launch_bounds__(RB) void reg_final_k(const double* __restrict__ part, int nblk, int P,
                                                  const float* __restrict__ g3,
                                                  float* __restrict__ out3, float* __restrict__ coef) {
  __shared__ double sh[RB / 64];
  __shared__ double tot[NPART];
  for (int k = 0; k < NPART; ++k) {
    double v = 0.0;
    for (int bI = threadIdx.x; bI < nblk; bI += RB) v += part[(size_t)k * RMAXB + bI];
    double t = block_sum(v, sh);
    if (threadIdx.x == 0) tot[k] = t;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const double numel = 3.0 * P * P, N = (double)P * P;
  const float nps = (float)(tot[0] / numel);
  const float tv = (float)((tot[1] + tot[2]) / numel);
  const double mu_rg = tot[3] / N, mu_yb = tot[4] / N;
  const double var_rg = (tot[5] - tot[3] * mu_rg) / (N - 1.0);   // torch.var: unbiased
  const double var_yb = (tot[6] - tot[4] * mu_yb) / (N - 1.0);
  const float sigma = sqrtf((float)var_rg + (float)var_yb);
  const float mu = sqrtf((float)(mu_rg * mu_rg) + (float)(mu_yb * mu_yb));
  out3[0] = nps;
  out3[1] = tv;
  out3[2] = sigma + 0.3f * mu;
  const float g_nps = g3 ? g3[0] : 0.f, g_tv = g3 ? g3[1] : 0.f, g_col = g3 ? g3[2] : 0.f;
  coef[0] = g_nps / (float)numel;
  coef[1] = g_tv / (float)numel;
  coef[2] = g_col;
  coef[3] = (float)mu_rg;
  coef[4] = (float)mu_yb;
  coef[5] = 0.5f / sigma * (2.f / (float)(N - 1.0));       // d sqrt(var_rg+var_yb) / d x_i = coef5*(x_i-mu)
  coef[6] = 0.3f * (float)mu_rg / mu / (float)N;            // d 0.3*sqrt(mu_rg^2+mu_yb^2) / d rg_i
  coef[7] = 0.3f * (float)mu_yb / mu / (float)N;
}

__device__ __forceinline__ float sgnf(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

// g3 != NULL: the upstream gradients are read here (coef[0..2] formed as
// reg_final_k forms them, from the statistics coef[3..7] of a forward
// po_regularisers call), so the backward is this one launch; acc: d += the
// gradient (one fp32 add of the complete value, as autograd sums two
// gradient contributions to the patch)
__global__ __launch_bounds__(RB) void reg_grad_k(const float* __restrict__ p, int P,
                                                 const float* __restrict__ col, int ncol,
                                                 const float* __restrict__ coef,
                                                 const float* __restrict__ g3, int acc,
                                                 float* __restrict__ d) {
  const int n = P * P;
  const int e = blockIdx.x * RB + threadIdx.x;
  if (e >= n) return;
  const size_t pp = (size_t)n;
  const int i = e / P, q = e % P;
  const float r = p[e], g = p[e + pp], b = p[e + 2 * pp];
  float dmin;
  int k;
  nps_pixel(col, ncol, r, g, b, dmin, k);
  const double numel = 3.0 * P * P;
  const float cn = g3 ? g3[0] / (float)numel : coef[0], ct = g3 ? g3[1] / (float)numel : coef[1],
              wc = g3 ? g3[2] : coef[2];
  const float rg = r - g, yb = 0.5f * (r + g) - b;
  const float drg = coef[5] * (rg - coef[3]) + coef[6];
  const float dyb = coef[5] * (yb - coef[4]) + coef[7];
  const float dcol[3] = {wc * (drg + 0.5f * dyb), wc * (-drg + 0.5f * dyb), wc * (-dyb)};
  const float pv[3] = {r, g, b};
  for (int ch = 0; ch < 3; ++ch) {
    const float* pc = p + ch * pp;
    float gn = cn * (pv[ch] - col[3 * k + ch] + 0.000001f) / dmin;
    float tvs = 0.f;
    if (q + 1 < P) tvs -= sgnf(pc[e + 1] - pc[e] + 0.000001f);
    if (q > 0) tvs += sgnf(pc[e] - pc[e - 1] + 0.000001f);
    if (i + 1 < P) tvs -= sgnf(pc[e + P] - pc[e] + 0.000001f);
    if (i > 0) tvs += sgnf(pc[e] - pc[e - P] + 0.000001f);
    const float v = gn + ct * tvs + dcol[ch];
    d[e + ch * pp] = acc ? d[e + ch * pp] + v : v;
  }
}
}  // namespace

extern "C" int po_regularisers(const float* patch, int P, const float* colors, int ncol, const float* g3,
                               float* out3, float* d_patch, float* workspace, po_stream_t s) {
  PO_REQUIRE(patch && colors && out3 && workspace, "po_regularisers: null pointer");
  PO_REQUIRE(P > 1 && ncol > 0, "po_regularisers: bad shape");
  PO_REQUIRE(!d_patch || g3, "po_regularisers: g3 required with d_patch");
  const int n = P * P;
  const int nblk = po::ceil_div(n, RB) < RMAXB ? po::ceil_div(n, RB) : RMAXB;
  double* part = reinterpret_cast<double*>(workspace);                   // 7*1024 doubles
  float* coef = workspace + 2 * NPART * RMAXB;                            // 8 floats
  hipStream_t st = po::stream_of(s);
  hipLaunchKernelGGL(reg_partial_k, dim3(nblk), dim3(RB), 0, st, patch, P, colors, ncol, part);
  int rc = po::check_launch("po_regularisers(partial)");
  if (rc) return rc;
  hipLaunchKernelGGL(reg_final_k, dim3(1), dim3(RB), 0, st, part, nblk, P, g3, out3, coef);
  rc = po::check_launch("po_regularisers(final)");
  if (rc || !d_patch) return rc;
  hipLaunchKernelGGL(reg_grad_k, dim3(po::ceil_div(n, RB)), dim3(RB), 0, st, patch, P, colors, ncol,
                     coef, nullptr, 0, d_patch);
  return po::check_launch("po_regularisers(grad)");
}

extern "C" int po_regularisers_grad(const float* patch, int P, const float* colors, int ncol, const float* g3,
                                    const float* workspace, int accumulate, float* d_patch, po_stream_t s) {
  PO_REQUIRE(patch && colors && g3 && workspace && d_patch, "po_regularisers_grad: null pointer");
  PO_REQUIRE(P > 1 && ncol > 0, "po_regularisers_grad: bad shape");
  const float* coef = workspace + 2 * NPART * RMAXB;      // the forward's statistics (coef[3..7])
  hipLaunchKernelGGL(reg_grad_k, dim3(po::ceil_div(P * P, RB)), dim3(RB), 0, po::stream_of(s), patch, P, colors,
                     ncol, coef, g3, accumulate ? 1 : 0, d_patch);
  return po::check_launch("po_regularisers_grad");
}
