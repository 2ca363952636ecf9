// Ablation microbenchmark of the po_conv main loop structure (tools only).
// 128x128 block tile, 4 waves x (2x2 32x32 tiles), BK=16 k-steps, fp32 MFMA.
// VARIANT: 1 = MFMA on registers only; 2 = + LDS fragment reads;
//          3 = + barrier per k-step; 4 = + LDS staging writes; 5 = + global loads.
// build: hipcc --offload-arch=gfx950 -O3 -DVARIANT=n tools/mfma_loop.hip -o /tmp/mfma_loop_n
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float floatx16 __attribute__((ext_vector_type(16)));
#ifndef VARIANT
#define VARIANT 5
#endif

__global__ __launch_bounds__(256) void loop_k(const float* __restrict__ A, const float* __restrict__ Bm,
                                              float* __restrict__ out, int nks) {
  constexpr int BM = 128, BN = 128, BK = 16, TM = 2, TN = 2;
  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * BK];
  float* As = smem;
  float* Bs = smem + 2 * BM * BK;
  const int tid = threadIdx.x & 255, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / 2, wn = wave % 2;
  const int cth = tid % 4, rth = tid / 4;
  floatx16 acc[TM][TN];
  for (int i = 0; i < TM; ++i)
    for (int j = 0; j < TN; ++j)
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  auto swz = [](int row, int chunk) { return (chunk ^ ((row >> 2) & 3)) * 4; };
  const float* ga = A + ((size_t)blockIdx.x * BM + rth) * 1024 + cth * 4;
  const float* gb = Bm + (size_t)rth * 1024 + cth * 4;
  float4 ra[2], rb[2];
  for (int r = 0; r < 2; ++r) {
    ra[r] = *reinterpret_cast<const float4*>(ga + r * 64 * 1024);
    rb[r] = *reinterpret_cast<const float4*>(gb + r * 64 * 1024);
  }
  for (int r = 0; r < 2; ++r) {
    *reinterpret_cast<float4*>(&As[(rth + 64 * r) * BK + swz(rth + 64 * r, cth)]) = ra[r];
    *reinterpret_cast<float4*>(&Bs[(rth + 64 * r) * BK + swz(rth + 64 * r, cth)]) = rb[r];
  }
  __syncthreads();
  const int arow = wm * 64 + (lane & 31), brow = wn * 64 + (lane & 31), h = lane >> 5;
  float4 af[TM], bf[TN];
  for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const float4*>(&As[(arow + 32 * i) * BK + swz(arow + 32 * i, h)]);
  for (int j = 0; j < TN; ++j) bf[j] = *reinterpret_cast<const float4*>(&Bs[(brow + 32 * j) * BK + swz(brow + 32 * j, h)]);
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = (VARIANT >= 4) ? (ks & 1) : 0;
    const float* Ab = As + buf * BM * BK;
    const float* Bb = Bs + buf * BN * BK;
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
#if VARIANT >= 2
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const float4*>(&Ab[(arow + 32 * i) * BK + swz(arow + 32 * i, 2 * g + h)]);
      for (int j = 0; j < TN; ++j)
        bf[j] = *reinterpret_cast<const float4*>(&Bb[(brow + 32 * j) * BK + swz(brow + 32 * j, 2 * g + h)]);
#endif
#if VARIANT >= 5
      if (g == 0) {
        const size_t koff = (size_t)((ks + 1) & 63) * 16;
        for (int r = 0; r < 2; ++r) {
          ra[r] = *reinterpret_cast<const float4*>(ga + r * 64 * 1024 + koff);
          rb[r] = *reinterpret_cast<const float4*>(gb + r * 64 * 1024 + koff);
        }
      }
#endif
      for (int i = 0; i < TM; ++i)
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i].x, bf[j].x, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i].y, bf[j].y, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i].z, bf[j].z, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i].w, bf[j].w, acc[i][j], 0, 0, 0);
        }
    }
#if VARIANT >= 4
    for (int r = 0; r < 2; ++r) {
      const int nb = buf ^ 1;
      *reinterpret_cast<float4*>(&As[(nb * BM + rth + 64 * r) * BK + swz(rth + 64 * r, cth)]) = ra[r];
      *reinterpret_cast<float4*>(&Bs[(nb * BN + rth + 64 * r) * BK + swz(rth + 64 * r, cth)]) = rb[r];
    }
#endif
#if VARIANT >= 3
    __syncthreads();
#endif
  }
  float s = 0.f;
  for (int i = 0; i < TM; ++i)
    for (int j = 0; j < TN; ++j)
      for (int e = 0; e < 16; ++e) s += acc[i][j][e];
  out[blockIdx.x * 256 + tid] = s;
}

__global__ void fill_k(float* p, size_t n, unsigned seed) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  unsigned x = (unsigned)i * 2654435761u + seed;
  x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
  p[i] = (float)(x & 0xffffff) / 16777216.0f * 2.0f - 1.0f;
}

int main(int argc, char** argv) {
  const int nblocks = argc > 1 ? atoi(argv[1]) : 1024;
  const int nks = argc > 2 ? atoi(argv[2]) : 256;
  float *A, *B, *O;
  hipMalloc(&A, (size_t)nblocks * 128 * 1024 * 4);
  hipMalloc(&B, (size_t)128 * 1024 * 4);
  hipMalloc(&O, (size_t)nblocks * 256 * 4);
  const int rnd = argc > 3 ? atoi(argv[3]) : 0;
  hipMemset(A, 0x3c, (size_t)nblocks * 128 * 1024 * 4);
  hipMemset(B, 0x3d, (size_t)128 * 1024 * 4);
  if (rnd) {
    const size_t na = (size_t)nblocks * 128 * 1024, nb = (size_t)128 * 1024;
    hipLaunchKernelGGL(fill_k, dim3((na + 255) / 256), dim3(256), 0, 0, A, na, 1u);
    hipLaunchKernelGGL(fill_k, dim3((nb + 255) / 256), dim3(256), 0, 0, B, nb, 7u);
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(loop_k, dim3(nblocks), dim3(256), 0, 0, A, B, O, nks);
  hipEventRecord(e0);
  const int it = 10;
  for (int w = 0; w < it; ++w) hipLaunchKernelGGL(loop_k, dim3(nblocks), dim3(256), 0, 0, A, B, O, nks);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= it;
  const double fl = 2.0 * nblocks * 128.0 * 128.0 * 16.0 * nks;
  printf("variant %d blocks %d nks %d rnd %d: %.1f us %.1f TFLOP/s\n", VARIANT, nblocks, nks, rnd, ms * 1e3,
         fl / ms / 1e9);
  return 0;
}
