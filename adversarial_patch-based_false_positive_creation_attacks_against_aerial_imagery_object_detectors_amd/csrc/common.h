// Shared helpers for libadvpatch_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
#include <map>
#include <mutex>
#include <utility>
#include "../../include/advpatch.h"

namespace po {

void set_error(const char* fmt, ...);

inline hipStream_t stream_of(po_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return PO_EHIP;
  }
  return PO_OK;
}

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// Workgroups of `kernel` the current device holds at once: its compute units
// times the resident workgroups per CU the occupancy calculator gives for this
// build (VGPRs, LDS, block size) -- the grid of a persistent kernel.
inline int resident_groups(const void* kernel, int block_threads, size_t dyn_lds = 0) {
  int dev = 0, cus = 0, occ = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                               hipSuccess)
    cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, block_threads, dyn_lds) != hipSuccess) occ = 1;
  return (cus > 0 ? cus : 1) * (occ > 0 ? occ : 1);
}

// resident_groups, remembered per (current device, kernel): a persistent
// launch queries the occupancy calculator once per device it runs on, so a
// process driving devices with different CU counts or partition modes sizes
// each device's grid from that device.
inline int resident_groups_cached(const void* kernel, int block_threads) {
  static std::mutex mu;
  static std::map<std::pair<int, const void*>, int> table;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  std::lock_guard<std::mutex> lock(mu);
  auto it = table.find({dev, kernel});
  if (it != table.end()) return it->second;
  const int n = resident_groups(kernel, block_threads);
  table[{dev, kernel}] = n;
  return n;
}

// leaky'(y) for LeakyReLU(0.1): PyTorch leaky_relu_backward uses x > 0
// (y and x share sign), slope 0.1 otherwise.
__device__ __forceinline__ float leaky_grad(float y) { return y > 0.f ? 1.f : 0.1f; }
// = (v > 0 ? v : 0.1 v), NaN and signed zeros included.  IEEE maximum (NaN-propagating,
// v_maximum3_f32 on gfx950): the same value as fmaxf for these operands (both NaN or
// neither, zeros of one sign) without the canonicalize fmaxf needs on a value the
// compiler cannot prove canonical (one VALU per element in the epilogues)
__device__ __forceinline__ float leaky(float v) { return __builtin_elementwise_maximum(v, v * 0.1f); }
// The activation of a conv epilogue without a branch on ConvArgs.act: slope 0.1
// is leaky() exactly, slope 1 the identity (maximum(v, v * 1) = v, NaN, signed
// zeros and infinities included) -- no per-element moves between the two paths.
__device__ __forceinline__ float act_slope(int act) { return act ? 0.1f : 1.0f; }

// OR of w over lanes i .. i+n-1 into lane i (n = 4 or 8, groups aligned inside
// a 16-lane DPP row; other lanes get partial ORs) by DPP row shifts
// (dst[i] = src[i + k], 0 past the row's end): VALU-rate, where __shfl_xor's
// dependent ds_bpermute round trips stall the epilogue.  Every lane of the
// wave must be active.
template <int n>
__device__ __forceinline__ uint32_t or_group_down(uint32_t w) {
  static_assert(n == 4 || n == 8, "groups of 4 or 8 lanes");
  w |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x101, 0xF, 0xF, false);   // row_shl:1
  w |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x102, 0xF, 0xF, false);   // row_shl:2
  if constexpr (n == 8) w |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x104, 0xF, 0xF, false);   // row_shl:4
  return w;
}
__device__ __forceinline__ float leaky_or_id(float v, float slope) { return __builtin_elementwise_maximum(v, v * slope); }

// torch.div(a, b, rounding_mode='floor') for float32 (ATen div_floor)
__device__ __forceinline__ float div_floor(float a, float b) {
  float mod = fmodf(a, b);
  float div = (a - mod) / b;
  if (mod != 0.f && ((b < 0.f) != (mod < 0.f))) div -= 1.f;
  float fl;
  if (div != 0.f) {
    fl = floorf(div);
    if (div - fl > 0.5f) fl += 1.f;
  } else {
    fl = copysignf(0.f, a / b);
  }
  return fl;
}

// Flat cell index of the patch centre (cx = column px, cy = row px) on a
// hw x hw head (train_patch.py:446-467; SURVEY Q1: index = ix*hw + iy).
// Sets *oob and clamps when the index leaves the map.
__device__ __forceinline__ int head_cell(float cx, float cy, int S, int hw, bool* oob) {
  const float stride = (float)((double)S / (double)hw);       // train_patch.py:446
  const int ix = (int)div_floor(cx, stride);                   // 449-450, 463
  const int iy = (int)div_floor(cy, stride);                   // 464
  int index = ix * hw + iy;                                    // 467
  *oob = index < 0 || index >= hw * hw;
  if (*oob) index = index < 0 ? 0 : hw * hw - 1;
  return index;
}

// Per-tensor max|x| slots of the split-precision (fp16x3) convolutions.  A
// slot is PO_AMAX_SUB uint32 sub-slots holding float bits (non-negative floats
// order like their bit patterns, so atomicMax on the bits is a float max); the
// bound of the tensor is the max over the sub-slots.  Writers spread over the
// sub-slots by workgroup and skip the atomic when the sub-slot already holds a
// larger value (a stale read only costs an extra atomic), so thousands of
// workgroups do not serialise on one address.  Every lane of the wave must
// call amax_commit (v >= 0).
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t u) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) u = max(u, (uint32_t)__shfl_xor((int)u, o));
  return u;
}

__device__ __forceinline__ void amax_commit(uint32_t* slot, float v) {
  const uint32_t u = wave_max_u32(__float_as_uint(v));
  if ((threadIdx.x & 63) == 0 && u) {
    uint32_t* s = slot + ((blockIdx.x + blockIdx.y * 7 + (threadIdx.x >> 6) * 13) & (PO_AMAX_SUB - 1));
    if (u > __atomic_load_n(s, __ATOMIC_RELAXED)) atomicMax(s, u);
  }
}

// max over the sub-slots (one load per lane), uniform across the wave
__device__ __forceinline__ uint32_t amax_read(const uint32_t* slot) {
  const uint32_t u = wave_max_u32(slot[threadIdx.x & (PO_AMAX_SUB - 1)]);
  return (uint32_t)__builtin_amdgcn_readfirstlane(u);
}

// XCD-aware bijective remap: consecutive logical tiles share an XCD's L2
// (workgroups are dispatched to the 8 XCDs round-robin: orig % 8)
__device__ __forceinline__ int xcd_remap() {
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  return (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + orig / 8;
}

}  // namespace po

#define PO_REQUIRE(cond, ...)          \
  do {                                 \
    if (!(cond)) {                     \
      po::set_error(__VA_ARGS__);      \
      return PO_EINVAL;                \
    }                                  \
  } while (0)
