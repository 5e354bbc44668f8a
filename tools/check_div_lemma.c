/* Exhaustive check of the f32 quotient lemma used by the narrow fast path
 * (DESIGN.md §Exactness):  for integers x >= 0, M >= 1 with 300*x + M < 2^24,
 *     floor(fl32(x * RU32(100/M))) == floor(100*x / M)
 * where RU32 is the smallest float >= 100/M and fl32 is IEEE single round-to-nearest.
 * Domain checked: every M in [1, MMAX], every x with 300x + M < 2^24 (and x <= XMAX).
 * Build: gcc -O2 -ffp-contract=off -o check_div_lemma check_div_lemma.c -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static float ru32_100_over(uint32_t M) {
  double r64 = 100.0 / (double)M;
  float f = (float)r64;
  if (fma((double)f, (double)M, -100.0) < 0.0) f = nextafterf(f, INFINITY);
  return f;
}

static uint64_t rng = 88172645463325252ull;
static uint64_t xorshift(void) { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return rng; }

int main(int argc, char** argv) {
  if (argc > 1 && argv[1][0] == 'r') {  /* random sample over the whole domain */
    uint64_t n = argc > 2 ? strtoull(argv[2], 0, 10) : 100000000ull, bad = 0;
    for (uint64_t i = 0; i < n; ++i) {
      uint32_t M = 1 + (uint32_t)(xorshift() % ((1u << 24) - 1));
      uint32_t xmax = (uint32_t)(((1ull << 24) - 1 - M) / 300);
      uint32_t x = (uint32_t)(xorshift() % ((uint64_t)xmax + 1));
      if ((i & 1) && xmax >= 64) x = xmax - (uint32_t)(xorshift() % 64); /* near the edge */
      volatile float p = (float)x * ru32_100_over(M);
      if ((uint32_t)p != (100ull * x) / M && bad++ < 5) printf("MISMATCH x=%u M=%u\n", x, M);
    }
    printf("random: %llu samples, %llu mismatches\n", (unsigned long long)n, (unsigned long long)bad);
    return bad != 0;
  }
  uint32_t MMAX = argc > 1 ? (uint32_t)atoi(argv[1]) : 60000;
  uint32_t XMAX = argc > 2 ? (uint32_t)atoi(argv[2]) : 60000;
  uint64_t checked = 0, bad = 0;
  for (uint32_t M = 1; M <= MMAX; ++M) {
    float r = ru32_100_over(M);
    if ((double)r < 100.0 / M - 1e-12) { printf("RU failed M=%u\n", M); return 2; }
    for (uint32_t x = 0; x <= XMAX && 300ull * x + M < (1ull << 24); ++x) {
      volatile float p = (float)x * r;
      uint32_t q = (uint32_t)p;
      uint64_t want = (100ull * x) / M;
      checked++;
      if (q != want) {
        if (bad++ < 5) printf("MISMATCH x=%u M=%u got %u want %llu\n", x, M, q,
                              (unsigned long long)want);
      }
    }
  }
  printf("checked %llu pairs, %llu mismatches\n", (unsigned long long)checked,
         (unsigned long long)bad);
  return bad != 0;
}
