// Pieces shared by the Winograd F(2x2,3x3) kernels of po_conv (conv_wino.hip:
// tiles 61, 65-68; conv_wino5.hip: tile 70).
#pragma once
#include "conv_common.h"

namespace {
using po::ConvArgs;

constexpr int WK = 16;   // input channels per k-step
constexpr uint32_t kOOB = 0x80000000u;     // an offset past every buffer resource's extent (< 2^31)
typedef float f2v __attribute__((ext_vector_type(2)));       // packed pairs: v_pk_add_f32

// tile-grid enumeration: GEMM row m -> image b, tile (ti, tj); with a.gbox
// only the tiles of the image's box (destination pixels [r0,r1) x [c0,c1))
__device__ __forceinline__ bool tile_point(const ConvArgs& a, int Ht, int Wt, int m, int& b, int& ti, int& tj) {
  const int per = Ht * Wt;
  b = ti = tj = 0;
  if (m >= a.B * per) return false;
  b = m / per;
  const int l = m - b * per;
  if (!a.gbox) {
    ti = l / Wt;
    tj = l - ti * Wt;
    return true;
  }
  const int4 bx = reinterpret_cast<const int4*>(a.gbox)[b];
  const int t0 = bx.x >> 1, t1 = (bx.z + 1) >> 1, u0 = bx.y >> 1, u1 = (bx.w + 1) >> 1;
  const int h = max(t1 - t0, 0), w = max(u1 - u0, 0);
  if (l >= h * w) return false;
  const int q = l / w;
  ti = t0 + q;
  tj = u0 + (l - q * w);
  return true;
}

__device__ __forceinline__ float4 f4add(float4 x, float4 y) { return make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w); }
__device__ __forceinline__ float4 f4sub(float4 x, float4 y) { return make_float4(x.x - y.x, x.y - y.y, x.z - y.z, x.w - y.w); }

// tile_point on a full map (no boxes): no memory access, no branch on a.gbox
__device__ __forceinline__ bool tile_point_full(const ConvArgs& a, int Ht, int Wt, int m, int& b, int& ti, int& tj) {
  const int per = Ht * Wt;
  const bool ok = m < a.B * per;
  b = ok ? m / per : 0;
  const int l = ok ? m - b * per : 0;
  ti = l / Wt;
  tj = l - ti * Wt;
  return ok;
}

// conv_wino4_k / conv_wino5_k: 64 2x2-tiles x 64 channels per workgroup; one
// transformed input buffer V[xi][tile][16 channels] (64 KB), 16-byte chunks
// swizzled by tile
constexpr int T4 = 64, N4 = 64;
constexpr int V4_FLOATS = 16 * T4 * WK;
__device__ __forceinline__ int v4idx(int xi, int t, int ch) { return ((xi * T4 + t) * WK) + ((ch ^ ((t >> 2) & 3)) << 2); }

// ---- persistent Winograd kernels (tiles 70, 71): buffer-resource helpers and
// the epilogue-field set
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
// tile_point_full with the two divisions by host magic numbers (ConvArgs
// mg_tiles / mg_wt): exact, and a multiply-high instead of a division sequence
// three times per unit
__device__ __forceinline__ bool tile_point_magic(const ConvArgs& a, int Ht, int Wt, int m, int& b, int& ti, int& tj) {
  const int per = Ht * Wt;
  const bool ok = m < a.B * per;
  b = ok ? po::div_by(m, a.mg_tiles, a.sh_tiles) : 0;
  const int l = ok ? m - b * per : 0;
  ti = po::div_by(l, a.mg_wt, a.sh_wt);
  tj = l - ti * Wt;
  return ok;
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float4 bld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ uint32_t bld1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}
__device__ __forceinline__ void bst4(float4 v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v), r, off, 0, 0);
}
__device__ __forceinline__ void bst1(uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 0);
}

// MODE 0's epilogue fields (one instantiation per combination the planner uses)
constexpr int EF_Y = 1;      // store y
constexpr int EF_RES = 2;    // load the shortcut operand, store the sum
constexpr int EF_ACC = 4;    // load the destination, accumulate
constexpr int EF_MB = 8;     // load the leaky-mask sign-bit word, multiply
constexpr int EF_Y2 = 16;    // load the second mask word, store the dual output
constexpr int EF_YB = 32;    // store the output's sign bits
constexpr int EF_POOL = 64;  // tile 71/72: the 2x2/2 max pool fused, only the pooled values and argmax bytes stored

}  // namespace
