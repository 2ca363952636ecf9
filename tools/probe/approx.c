/* Hardware reciprocal-square-root approximations of the host CPU over every
 * fp32 in [1, 4) (two binades: both exponent parities), written as uint32
 * bit patterns: rsqrt14 (AVX-512) then rsqrt (AVX, 12-bit), rcp14, rcp.
 * Input to tools/sqrt_probe.py's search for MKL VML's vsSqrt algorithm.
 * gcc -O2 -mavx512f -mavx2 -mfma approx.c -o approx */
#include <immintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
int main(int argc, char** argv) {
  const uint32_t n = 1u << 24;
  uint32_t* out = (uint32_t*)malloc((size_t)n * 4);
  const char* names[4] = {"rsqrt14", "rsqrt", "rcp14", "rcp"};
  for (int f = 0; f < 4; ++f) {
    for (uint32_t i = 0; i < n; i += 16) {
      uint32_t bits[16];
      for (int l = 0; l < 16; ++l) bits[l] = 0x3F800000u + i + l;   /* 1.0 .. 4.0 */
      __m512 x;
      memcpy(&x, bits, 64);
      __m512 y;
      if (f == 0) y = _mm512_rsqrt14_ps(x);
      else if (f == 2) y = _mm512_rcp14_ps(x);
      else {
        __m256 lo, hi;
        memcpy(&lo, bits, 32);
        memcpy(&hi, bits + 8, 32);
        lo = f == 1 ? _mm256_rsqrt_ps(lo) : _mm256_rcp_ps(lo);
        hi = f == 1 ? _mm256_rsqrt_ps(hi) : _mm256_rcp_ps(hi);
        memcpy(bits, &lo, 32);
        memcpy(bits + 8, &hi, 32);
        memcpy(&y, bits, 64);
      }
      memcpy(out + i, &y, 64);
    }
    char path[512];
    snprintf(path, sizeof(path), "%s/%s.u32", argc > 1 ? argv[1] : ".", names[f]);
    FILE* fp = fopen(path, "wb");
    fwrite(out, 4, n, fp);
    fclose(fp);
  }
  free(out);
  return 0;
}
