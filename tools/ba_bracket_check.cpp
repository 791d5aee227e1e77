// Check of the resource-only sweep's fraction bracket (ksched_eval.hpp,
// DESIGN.md §4): with y = RN(1/Allocatable), ry = RN(Requested * y) and
// q = fma(request, y, ry) per resource,
//   * Fit:  Requested + request <= Allocatable  iff  q <= 1 + 2^-49
//     (Allocatable != 0; a request of 0 skips the check);
//   * BalancedAllocation: with v± = fma(|q_cpu - q_mem|, -50, 100 ± 2^-40),
//     trunc(v-) == trunc(v+) implies it equals upstream's
//     int64((1 - |(f_cpu - f_mem) / 2|) * 100), f = min(1, (Requested +
//     request) / Allocatable) as IEEE binary64 quotients (balanced_allocation.go),
//     on feasible nodes whose Requested <= Allocatable with both allocatables
//     non-zero (the others are fixed or recomputed exactly by the sweep).
// Reports the undecided share (the sweep's exact-recompute rate).
// Build: g++ -O2 -mfma -ffp-contract=off ba_bracket_check.cpp
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>

static const double FIT_Q_MAX = 1.0 + 0x1p-49;
static const double BA_LO = 100.0 - 0x1p-40, BA_HI = 100.0 + 0x1p-40;

static uint64_t n_fit = 0, bad_fit = 0, n_ba = 0, bad_ba = 0, undecided = 0;

static int64_t ba_exact(int64_t ac, int64_t am, int64_t sc, int64_t sm) {
  double f0 = std::fmin(1.0, (double)sc / (double)ac), f1 = std::fmin(1.0, (double)sm / (double)am);
  double sd = std::fabs((f0 - f1) / 2);
  return (int64_t)((1 - sd) * 100.0);
}

static void test(int64_t ac, int64_t am, int64_t rc, int64_t rm, int64_t qc, int64_t qm) {
  const double yc = ac ? 1.0 / (double)ac : 0.0, ym = am ? 1.0 / (double)am : 0.0;
  const double ryc = (double)rc * yc, rym = (double)rm * ym;
  const double q0 = std::fma((double)qc, yc, ryc), q1 = std::fma((double)qm, ym, rym);
  // Fit, per resource with a request
  const bool fit_c = qc == 0 || (ac != 0 && !(q0 > FIT_Q_MAX)), fit_m = qm == 0 || (am != 0 && !(q1 > FIT_Q_MAX));
  const bool ex_c = qc == 0 || rc + qc <= ac, ex_m = qm == 0 || rm + qm <= am;
  ++n_fit;
  if (fit_c != ex_c || fit_m != ex_m) {
    if (bad_fit < 10)
      printf("FIT MISMATCH ac=%lld rc=%lld qc=%lld am=%lld rm=%lld qm=%lld\n", (long long)ac, (long long)rc,
             (long long)qc, (long long)am, (long long)rm, (long long)qm);
    ++bad_fit;
  }
  if (!(ex_c && ex_m) || ac == 0 || am == 0 || rc > ac || rm > am) return;
  const double ad = std::fabs(q0 - q1);
  const double vlo = std::fma(ad, -50.0, BA_LO), vhi = std::fma(ad, -50.0, BA_HI);
  const int64_t lo = (int64_t)vlo, hi = (int64_t)vhi;
  ++n_ba;
  if (lo != hi) {
    ++undecided;
    return;
  }
  const int64_t want = ba_exact(ac, am, rc + qc, rm + qm);
  if (hi != want) {
    if (bad_ba < 10)
      printf("BA MISMATCH ac=%lld rc=%lld qc=%lld am=%lld rm=%lld qm=%lld got=%lld want=%lld\n", (long long)ac,
             (long long)rc, (long long)qc, (long long)am, (long long)rm, (long long)qm, (long long)hi,
             (long long)want);
    ++bad_ba;
  }
}

int main() {
  std::mt19937_64 g(7);
  auto below = [&](int64_t n) -> int64_t { return n > 0 ? (int64_t)(g() % (uint64_t)n) : 0; };
  const int64_t Mi = 1ll << 20, Gi = 1ll << 30;
  const int64_t cpus[] = {8000, 16000, 32000, 64000, 96000};
  const int64_t mems[] = {32 * Gi, 64 * Gi, 128 * Gi, 256 * Gi, 512 * Gi};
  // 1. the synthetic shapes: cpu in 50m steps, memory in 64Mi steps, with
  //    sums landing exactly on the allocatable
  for (int k = 0; k < 20000000; ++k) {
    const int64_t ac = cpus[below(5)], am = mems[below(5)];
    const int64_t rc = 50 * below(ac / 50 + 1), rm = 64 * Mi * below(am / (64 * Mi) + 1);
    int64_t qc = 50 * below(81), qm = 64 * Mi * below(257);
    if (k % 7 == 0) qc = ac - rc;  // exactly full
    if (k % 11 == 0) qm = am - rm;
    if (k % 13 == 0) qc = 0;
    if (k % 17 == 0) qm = 0;
    test(ac, am, rc, rm, qc, qm);
  }
  // 2. random magnitudes: allocatables up to 2^44 (the upsert bound)
  for (int k = 0; k < 20000000; ++k) {
    const int64_t ac = 1 + below((1ll << (1 + below(44))) - 1), am = 1 + below((1ll << (1 + below(44))) - 1);
    const int64_t rc = below(ac + 1), rm = below(am + 1);
    int64_t qc = below(2 * (ac - rc) + 2), qm = below(2 * (am - rm) + 2);
    if (k % 5 == 0) qc = ac - rc + below(3) - 1;  // at and around the boundary
    if (k % 9 == 0) qm = am - rm + below(3) - 1;
    if (qc < 0) qc = 0;
    if (qm < 0) qm = 0;
    test(ac, am, rc, rm, qc, qm);
  }
  // 3. equal fractions (std = 0), halves and near-equal ratios
  for (int k = 0; k < 5000000; ++k) {
    const int64_t ac = cpus[below(5)], am = mems[below(5)];
    const int64_t t = 1 + below(64);
    const int64_t sc = ac / 64 * t, sm = am / 64 * (k % 3 == 0 ? t : (t + below(3) - 1 + 64) % 65);
    const int64_t rc = below(sc + 1), rm = below(sm + 1);
    test(ac, am, rc, rm, sc - rc, sm - rm);
  }
  // 4. overcommitted / zero allocatables (Fit only)
  for (int k = 0; k < 2000000; ++k) {
    const int64_t ac = below(3) ? cpus[below(5)] : 0, am = below(3) ? mems[below(5)] : 0;
    test(ac, am, below(2 * ac + 2), below(2 * am + 2), below(2000), below(4 * Gi));
  }
  printf("checked fit %llu, ba %llu (undecided %llu = %.3g), mismatches %llu\n", (unsigned long long)n_fit,
         (unsigned long long)n_ba, (unsigned long long)undecided, n_ba ? (double)undecided / (double)n_ba : 0.0,
         (unsigned long long)(bad_fit + bad_ba));
  return (bad_fit + bad_ba) != 0;
}
