// Exhaustive check of warp_geom.h ref_base: fl(x / S) == fma(fma(-q, S, x), rcp, q),
// q = fl(x rcp), rcp = fl(1/S), x = fl(linspace_k * (S-1)), for every k < S, S <= 32768.
// gcc -O2 -ffp-contract=off -o /tmp/markstein tools/probe/markstein_check.c -lm
#include <stdio.h>
#include <math.h>
#include <string.h>
int main(void) {
  long bad = 0, n = 0;
  for (int S = 2; S <= 32768; ++S) {
    volatile float fS = (float)S, fS1 = (float)(S - 1);
    const float step = 2.0f / fS1, y = 1.0f / fS;
    for (int k = 0; k < S; ++k) {
      const float lin = k < (S >> 1) ? fmaf(step, (float)k, -1.0f) : fmaf(-step, (float)(S - 1 - k), 1.0f);
      const float x = lin * fS1;
      const float want = x / fS;
      const float q = x * y;
      const float r = fmaf(-q, fS, x);
      const float b = fmaf(r, y, q);
      ++n;
      if (memcmp(&b, &want, 4)) { if (bad < 5) printf("S=%d k=%d x=%a want=%a got=%a\n", S, k, x, want, b); ++bad; }
    }
  }
  printf("%ld of %ld differ\n", bad, n);
  return 0;
}
