// Exhaustive check behind as_secs_f64 (ruserf_amd/csrc/common.h): for every integer x in
// [0, 1e9) -- the whole domain of Duration nanos -- q0 = x * RN(1e-9) followed by one FMA
// correction, fma(fma(-q0, 1e9, x), RN(1e-9), q0), equals the correctly rounded x / 1e9.
#include <math.h>
#include <stdio.h>
#include <stdint.h>
int main(void) {
  const double R = 1.0 / 1e9, D = 1e9;
  uint64_t bad = 0, first = 0;
  for (uint32_t x = 0; x < 1000000000u; ++x) {
    const double xd = (double)x;
    const double ref = xd / D;
    const double q0 = xd * R;
    const double e = fma(-q0, D, xd);
    const double q1 = fma(e, R, q0);
    if (q1 != ref) { if (!bad) first = x; ++bad; }
  }
  printf("R=%.17g bad=%llu first=%llu\n", R, (unsigned long long)bad, (unsigned long long)first);
  return bad != 0;
}
