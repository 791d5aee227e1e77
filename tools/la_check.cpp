// LeastAllocated exactness check for the sweep's truncation formula
// (ksched_kernels.hip least_requested):
//   floor(x / cap) == (int) fma(x, RN(1/cap), 2^-45)   for x = r * 100,
//   1 <= cap < 2^44, 0 <= r <= cap  (r = capacity - requested, clamped >= 0).
// Covers every r for small capacities, quotients next to every integer
// k = 0..100 for random capacities (the adversarial cases: fractional part 0,
// 1/cap or 1 - 1/cap), capacities next to powers of two and 2^44 - 1.
// Build: g++ -O2 -mfma -ffp-contract=off la_check.cpp -o la_check
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>
int main() {
  std::mt19937_64 g(7);
  uint64_t bad = 0, n = 0;
  auto test = [&](int64_t r, int64_t cap) {
    if (r < 0 || r > cap) return;
    const uint64_t x = (uint64_t)r * 100u;
    const int64_t want = (int64_t)(x / (uint64_t)cap);
    const double y = 1.0 / (double)cap;
    const int64_t got = (int64_t)std::fma((double)x, y, 0x1p-45);
    ++n;
    if (got != want) {
      if (bad < 10) printf("MISMATCH r=%lld cap=%lld want=%lld got=%lld\n", (long long)r, (long long)cap,
                           (long long)want, (long long)got);
      ++bad;
    }
  };
  for (int64_t cap = 1; cap <= 2000; ++cap)
    for (int64_t r = 0; r <= cap; ++r) test(r, cap);
  for (int64_t cap : {8000ll, 16000ll, 32000ll, 64000ll, 96000ll, 100000ll, 128000ll, 192000ll})
    for (int64_t r = 0; r <= cap; ++r) test(r, cap);
  auto near_integers = [&](int64_t cap) {
    for (int64_t k = 0; k <= 100; ++k) {
      // r with r*100 closest to k*cap from both sides
      const int64_t r0 = (int64_t)(((__int128)k * cap) / 100);
      for (int64_t d = -3; d <= 3; ++d) test(r0 + d, cap);
    }
    test(cap, cap);
    test(0, cap);
  };
  for (int i = 0; i < 2000000; ++i) {
    const int sh = (int)(g() % 44);
    int64_t cap = (int64_t)(g() >> (64 - 44)) >> sh;
    if (cap < 1) cap = 1;
    near_integers(cap);
    for (int j = 0; j < 4; ++j) test((int64_t)(g() % (uint64_t)(cap + 1)), cap);
  }
  for (int e = 1; e <= 44; ++e)
    for (int64_t d = -50; d <= 50; ++d) {
      const int64_t cap = (1ll << e) + d;
      if (cap >= 1 && cap < (1ll << 44)) near_integers(cap);
    }
  const int64_t Gi = 1ll << 30;
  for (int64_t cap : {32 * Gi, 64 * Gi, 128 * Gi, 256 * Gi, 512 * Gi, 1024 * Gi, 16383 * Gi})
    for (int64_t r = 0; r <= cap; r += 1 << 20) test(r, cap);
  printf("checked %llu, mismatches %llu\n", (unsigned long long)n, (unsigned long long)bad);
  return bad != 0;
}
