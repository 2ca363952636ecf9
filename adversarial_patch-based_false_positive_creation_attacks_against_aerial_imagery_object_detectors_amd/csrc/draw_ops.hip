// Per-step random draws of the patch transformer and the patch-gradient
// finiteness guard.
//
// po_draws replaces the reference's draws (load_data.py:548-574 contrast /
// brightness / noise from the CUDA RNG, 607-614 angle, 693-707 target_x/y from
// the CPU RNG) with a counter-based generator: every variate is a pure
// function of (seed, step counter, GLOBAL image index, element), so a rank
// that processes images [b0, b0+B) of a global batch draws exactly the rows
// a single process would draw for them — the data-parallel result does not
// depend on the number of ranks and a step needs no host RNG.
//
// Generator: Philox4x32-10 (Salmon et al., SC'11), key = seed, counter =
// {element group, global image, step lo, step hi}; one call gives 4 uniform
// u = (x >> 8) * 2^-24 in [0,1).  Noise element e of image b is lane e%4 of
// group e/4; the per-image scalars are groups 0xFFFFFFFF {contrast, bright,
// angle, ux} and 0xFFFFFFFE {uy}.  oracle/draws_ref.py restates it in numpy.
#pragma clang fp contract(off)
#include "common.h"
#include "philox.h"

namespace {

using po::u4;
using po::philox4x32_10;
__device__ __forceinline__ float unif(uint32_t x) { return po::philox_unif(x); }
__device__ __forceinline__ float affine(float u, float span, float from) { return po::philox_affine(u, span, from); }

constexpr float kPi = 3.14159265358979323846f;

__global__ __launch_bounds__(256) void draws_k(uint32_t k0, uint32_t k1, uint32_t c_lo, uint32_t c_hi, int b0,
                                               int n, float* __restrict__ contrast, float* __restrict__ bright,
                                               float* __restrict__ noise, float* __restrict__ angle,
                                               float* __restrict__ ux, float* __restrict__ uy) {
  const int b = blockIdx.y;
  const uint32_t gb = (uint32_t)(b0 + b);
  const int g = blockIdx.x * 256 + threadIdx.x;        // element group of 4 noise values
  const int ngroups = (n + 3) / 4;
  if (g < ngroups && noise) {
    const u4 r = philox4x32_10(u4{(uint32_t)g, gb, c_lo, c_hi}, k0, k1);
    float* o = noise + (size_t)b * n;
    const float v[4] = {affine(unif(r.x), 2.0f, -1.0f), affine(unif(r.y), 2.0f, -1.0f),
                        affine(unif(r.z), 2.0f, -1.0f), affine(unif(r.w), 2.0f, -1.0f)};
    const int e0 = 4 * g;
    if (e0 + 4 <= n && (n & 3) == 0) {
      *reinterpret_cast<float4*>(o + e0) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      for (int q = 0; q < 4 && e0 + q < n; ++q) o[e0 + q] = v[q];
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const u4 s = philox4x32_10(u4{0xFFFFFFFFu, gb, c_lo, c_hi}, k0, k1);
    const u4 t = philox4x32_10(u4{0xFFFFFFFEu, gb, c_lo, c_hi}, k0, k1);
    if (contrast) contrast[b] = affine(unif(s.x), 0.4f, 0.8f);      // U(0.8, 1.2)   load_data.py:548-553
    if (bright) bright[b] = affine(unif(s.y), 0.2f, -0.1f);         // U(-0.1, 0.1)  556-561
    if (angle) angle[b] = affine(unif(s.z), 2.0f * kPi, -kPi);      // U(-pi, pi)    607-614
    if (ux) ux[b] = unif(s.w);                                       // U(0,1)        693-707
    if (uy) uy[b] = unif(t.x);
  }
}

// flags[0] |= bit if any of x[0..n) is NaN or +-Inf
__global__ __launch_bounds__(256) void check_finite_k(const float* __restrict__ x, int64_t n, int32_t bit,
                                                      int32_t* __restrict__ flags) {
  bool bad = false;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    bad |= !isfinite(x[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flags, bit);
}

// found_inf = 1.0f while the bit is up (after check_finite_k on the same stream)
__global__ void found_inf_k(const int32_t* __restrict__ flags, int32_t bit, float* __restrict__ found_inf) {
  *found_inf = (*flags & bit) ? 1.f : 0.f;
}

// Adam(amsgrad) + clamp, one thread per element, in torch.optim.Adam's
// single-tensor order (torch/optim/adam.py, the reference's CPU arithmetic):
// exp_avg.lerp_(g, 1 - beta1) (ATen's vectorised lerp: fma(w, g - m, m)),
// exp_avg_sq.mul_(beta2).addcmul_(g, g, value=1 - beta2), torch.maximum into
// max_exp_avg_sq, denom = sqrt(max) / sqrt(1 - beta2^t) + eps, param +=
// (-lr / (1 - beta1^t)) * exp_avg / denom, then clamp_(lo, hi) (NaN kept).
// The scalars are formed in float64 from the step count t = step_in + 1, as
// the Python floats of the reference; a raised found_inf / flag bit skips the
// update and leaves the count (PyTorch's fused-Adam found_inf contract).
// step_out != step_in (the caller alternates two counters): no block reads a
// count another block writes.
__global__ __launch_bounds__(256) void adam_amsgrad_k(float* __restrict__ p, const float* __restrict__ g,
                                                      float* __restrict__ m, float* __restrict__ v,
                                                      float* __restrict__ vmax, int64_t n,
                                                      const float* __restrict__ step_in, float* __restrict__ step_out,
                                                      double lr, double beta1, double beta2, float w1, float b2,
                                                      float w2, float eps, const float* __restrict__ found_inf,
                                                      const int32_t* __restrict__ flags, int32_t bit, int clamp,
                                                      float lo, float hi) {
  const bool skip = (found_inf && *found_inf != 0.f) || (flags && (*flags & bit));
  const float s0 = *step_in;
  if (blockIdx.x == 0 && threadIdx.x == 0) *step_out = skip ? s0 : s0 + 1.f;
  if (skip) return;
  const double t = (double)(s0 + 1.f);
  const float neg_step = (float)(-(lr / (1.0 - pow(beta1, t))));
  const float bc2s = (float)sqrt(1.0 - pow(beta2, t));
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float gi = g[i];
    const float mi = __builtin_fmaf(w1, gi - m[i], m[i]);
    float vi = v[i] * b2;
    vi = vi + (w2 * gi) * gi;
    const float vm = __builtin_elementwise_maximum(vmax[i], vi);
    const float denom = sqrtf(vm) / bc2s + eps;
    float pi = p[i] + (neg_step * mi) / denom;
    if (clamp && !isnan(pi)) pi = fminf(fmaxf(pi, lo), hi);
    m[i] = mi;
    v[i] = vi;
    vmax[i] = vm;
    p[i] = pi;
  }
}

}  // namespace

extern "C" int po_adam_amsgrad(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                               float* max_exp_avg_sq, int64_t n, const float* step_in, float* step_out, double lr,
                               double beta1, double beta2, double eps, const float* found_inf,
                               const int32_t* flags, int32_t bit, int clamp, float lo, float hi, po_stream_t s) {
  PO_REQUIRE(param && grad && exp_avg && exp_avg_sq && max_exp_avg_sq && step_in && step_out && n >= 0,
             "po_adam_amsgrad: null pointer");
  PO_REQUIRE(step_in != step_out, "po_adam_amsgrad: step_in and step_out must differ");
  PO_REQUIRE(beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0 && eps >= 0.0,
             "po_adam_amsgrad: bad hyper-parameters");
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(po::ceil_div(n, 256), 2048));
  hipLaunchKernelGGL(adam_amsgrad_k, dim3(grid), dim3(256), 0, po::stream_of(s), param, grad, exp_avg, exp_avg_sq,
                     max_exp_avg_sq, n, step_in, step_out, lr, beta1, beta2, (float)(1.0 - beta1), (float)beta2,
                     (float)(1.0 - beta2), (float)eps, found_inf, flags, bit, clamp, lo, hi);
  return po::check_launch("po_adam_amsgrad");
}

extern "C" int po_draws(uint64_t seed, uint64_t counter, int b0, int B, int P, float* contrast, float* bright,
                        float* noise, float* angle, float* ux, float* uy, po_stream_t s) {
  PO_REQUIRE(B >= 1 && B <= 65535 && b0 >= 0 && P >= 1, "po_draws: bad sizes (b0=%d B=%d P=%d)", b0, B, P);
  const int64_t n = 3LL * P * P;
  PO_REQUIRE(n < (1LL << 31), "po_draws: patch too large");
  const int ngroups = (int)((n + 3) / 4);
  dim3 grid(noise ? po::ceil_div(ngroups, 256) : 1, B);
  hipLaunchKernelGGL(draws_k, grid, dim3(256), 0, po::stream_of(s), (uint32_t)seed, (uint32_t)(seed >> 32),
                     (uint32_t)counter, (uint32_t)(counter >> 32), b0, (int)n, contrast, bright, noise, angle, ux,
                     uy);
  return po::check_launch("po_draws");
}

extern "C" int po_check_finite_inf(const float* x, int64_t n, int32_t bit, int32_t* flags, float* found_inf,
                                  po_stream_t s) {
  PO_REQUIRE(x && flags && n >= 0, "po_check_finite: null pointer");
  if (n == 0) {
    if (found_inf) hipLaunchKernelGGL(found_inf_k, dim3(1), dim3(1), 0, po::stream_of(s), flags, bit, found_inf);
    return po::check_launch("po_check_finite");
  }
  const int grid = (int)std::min<int64_t>(po::ceil_div(n, 256), 1024);
  hipLaunchKernelGGL(check_finite_k, dim3(grid), dim3(256), 0, po::stream_of(s), x, n, bit, flags);
  if (found_inf) hipLaunchKernelGGL(found_inf_k, dim3(1), dim3(1), 0, po::stream_of(s), flags, bit, found_inf);
  return po::check_launch("po_check_finite");
}

extern "C" int po_check_finite(const float* x, int64_t n, int32_t bit, int32_t* flags, po_stream_t s) {
  return po_check_finite_inf(x, n, bit, flags, nullptr, s);
}
