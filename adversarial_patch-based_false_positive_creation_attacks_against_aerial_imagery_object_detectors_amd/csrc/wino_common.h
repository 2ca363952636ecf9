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
}  // namespace
