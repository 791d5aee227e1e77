// Exhaustive-ish check: for b = allocatable (integer, 1 <= b < 2^46) and
// a = requested (integer, 0 <= a < 2^47), is  q1 = fma(fma(-b,q0,a), y, q0)
// with y = RN(1/b), q0 = RN(a*y)  equal to the IEEE quotient RN(a/b)?
// Build: g++ -O2 -mfma -ffp-contract=off markstein_check.cpp
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>
static inline double mq(double a, double b, double y) {
  double q0 = a * y;
  double r = std::fma(-b, q0, a);
  return std::fma(r, y, q0);
}
int main(int argc, char **argv) {
  std::mt19937_64 g(42);
  uint64_t bad = 0, n = 0;
  auto test = [&](int64_t ai, int64_t bi) {
    double a = (double)ai, b = (double)bi, y = 1.0 / b;
    double q = a / b, m = mq(a, b, y);
    ++n;
    if (q != m) { if (bad < 10) printf("MISMATCH a=%lld b=%lld q=%.17g m=%.17g\n", (long long)ai, (long long)bi, q, m); ++bad; }
  };
  const int64_t cpus[] = {8000, 16000, 32000, 64000, 96000, 1000, 3, 7, 999, 100000};
  for (int64_t b : cpus) for (int64_t a = 0; a <= 4 * b; ++a) test(a, b);          // every cpu request
  for (int k = 0; k < 60000000; ++k) {                                             // memory-like
    int64_t b = (int64_t)(g() % ((1ull << 46) - 1)) + 1;
    int sh = g() % 47; if (sh) b = std::max<int64_t>(1, b >> sh);
    int64_t a = (int64_t)(g() % (uint64_t)(2 * b + 1));
    test(a, b);
  }
  for (int e = 1; e < 46; ++e) for (int d = -3; d <= 3; ++d) {                       // near powers of two
    int64_t b = (1ll << e) + d; if (b <= 0) continue;
    for (int k = 0; k < 20000; ++k) test((int64_t)(g() % (uint64_t)(2 * b + 1)), b);
  }
  const int64_t Gi = 1ll << 30;
  for (int64_t b : {32 * Gi, 64 * Gi, 128 * Gi, 256 * Gi, 512 * Gi})                  // 64Mi granularity sums
    for (int64_t a = 0; a <= b; a += 1 << 20) test(a, b);
  printf("checked %llu, mismatches %llu\n", (unsigned long long)n, (unsigned long long)bad);
  return bad != 0;
}
