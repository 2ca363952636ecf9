// Philox4x32-10 counter-based generator (Salmon et al., SC'11) shared by
// po_draws (draw_ops.hip) and the warp kernels that regenerate the
// transformer's noise in-kernel (patch_ops.hip): key = seed, counter =
// {element group, global image, step lo, step hi}; one call gives 4 uniform
// u = (x >> 8) * 2^-24 in [0,1).  oracle/draws_ref.py restates it in numpy.
// Include after `#pragma clang fp contract(off)`.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace po {

struct u4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ u4 philox4x32_10(u4 c, uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32x32 -> 64-bit product per word (v_mad_u64_u32) instead of a
    // separate low and high multiply (both quarter-rate)
    const uint64_t p0 = (uint64_t)M0 * c.x, p1 = (uint64_t)M1 * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    c = u4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

__device__ __forceinline__ float philox_unif(uint32_t x) { return (float)(x >> 8) * 0x1p-24f; }
// from + u * span for fp32 u, span, from: the product is exact in float64
// (24 + 24 bits), so the float64 sum is rounded once and then to fp32 — the
// same bits whether or not the compiler fuses the multiply-add
__device__ __forceinline__ float philox_affine(float u, float span, float from) {
  return (float)((double)u * (double)span + (double)from);
}

// Noise element e (flat over [3][P][P]) of global image gb at step (c_lo, c_hi):
// U(-1, 1), lane e % 4 of group e / 4 (load_data.py:566-568; x0.1 by the caller)
__device__ __forceinline__ float philox_noise(uint32_t k0, uint32_t k1, uint32_t c_lo, uint32_t c_hi, uint32_t gb,
                                              uint32_t e) {
  const u4 r = philox4x32_10(u4{e >> 2, gb, c_lo, c_hi}, k0, k1);
  const uint32_t l = e & 3u;
  const uint32_t x = l == 0 ? r.x : (l == 1 ? r.y : (l == 2 ? r.z : r.w));
  return philox_affine(philox_unif(x), 2.0f, -1.0f);
}

}  // namespace po
