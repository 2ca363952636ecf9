// Shared helpers for libadvpatch_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
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

// leaky'(y) for LeakyReLU(0.1): PyTorch leaky_relu_backward uses x > 0
// (y and x share sign), slope 0.1 otherwise.
__device__ __forceinline__ float leaky_grad(float y) { return y > 0.f ? 1.f : 0.1f; }
__device__ __forceinline__ float leaky(float v) { return v > 0.f ? v : v * 0.1f; }

}  // namespace po

#define PO_REQUIRE(cond, ...)          \
  do {                                 \
    if (!(cond)) {                     \
      po::set_error(__VA_ARGS__);      \
      return PO_EINVAL;                \
    }                                  \
  } while (0)
