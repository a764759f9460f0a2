/* Exhaustive check behind div1000() (reporter_amd/csrc/otr_kernels.h, used by k_viterbi):
 * for every integral x in [0, 2^32), fma(fma(-RN(x*0.001), 1000, x), 0.001, RN(x*0.001))
 * equals the correctly rounded quotient x / 1000.0.  Prints the mismatch count. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>

int main(void) {
  uint64_t bad = 0;
  for (uint64_t r = 0; r <= 0xFFFFFFFFull; ++r) {
    const double x = (double)r;
    const double q0 = x * 0.001;
    const double q1 = fma(fma(-q0, 1000.0, x), 0.001, q0);
    if (q1 != x / 1000.0) ++bad;
  }
  printf("%llu\n", (unsigned long long)bad);
  return 0;
}
