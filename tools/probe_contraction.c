/* probe_contraction.c -- which product of d.x*d.x + d.y*d.y + d.z*d.z (simple_knn.cu:136's expression)
 * a compiler fuses under FMA contraction.  Build and run (DESIGN.md "Parity"):
 *   clang -O2 -ffp-contract=fast -mfma tools/probe_contraction.c -lm && ./a.out    (also -ffp-contract=on, gcc)
 * Every build here fuses the LEFT product: fmaf(dz, dz, fmaf(dx, dx, dy * dy)); the two candidate forms
 * differ on ~15% of random inputs. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
__attribute__((noinline)) float expr(float dx, float dy, float dz) { return dx * dx + dy * dy + dz * dz; }
int main() {
  srand(1); int a = 0, b = 0, both = 0, n = 10000000;
  for (int i = 0; i < n; i++) {
    float dx = (rand() / (float)RAND_MAX - 0.5f) * 3, dy = (rand() / (float)RAND_MAX - 0.5f) * 3, dz = (rand() / (float)RAND_MAX - 0.5f) * 3;
    float e = expr(dx, dy, dz);
    float A = fmaf(dz, dz, fmaf(dx, dx, dy * dy));  // left product fused
    float B = fmaf(dz, dz, fmaf(dy, dy, dx * dx));  // right product fused
    int ea = memcmp(&e, &A, 4) == 0, eb = memcmp(&e, &B, 4) == 0;
    a += ea && !eb; b += eb && !ea; both += ea && eb;
  }
  printf("matches only fma(dz,dz,fma(dx,dx,dy*dy)): %d, only fma(dz,dz,fma(dy,dy,dx*dx)): %d, both: %d of %d\n", a, b, both, n);
}
