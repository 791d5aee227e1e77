// ksched_sort.hip — device radix sort of (64-bit key, 32-bit value) pairs
// (hipCUB over rocPRIM), kept in its own translation unit: the replica runs of
// the spread path (ksched_spread.hip) order a run's feasible
// nodes by (group, static score descending, slot) once per run, carrying each
// node's position.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "ksched_kernels.hpp"

namespace ks {

// tmp == nullptr: *tmp_bytes = the scratch a sort of n pairs needs.
// Stable: equal keys keep their input order.  Bits [0, end_bit) are sorted.
hipError_t launch_sort_pairs(const uint64_t *kin, uint64_t *kout, const uint32_t *vin, uint32_t *vout, uint32_t n,
                             uint32_t end_bit, void *tmp, size_t *tmp_bytes, hipStream_t st) {
  return hipcub::DeviceRadixSort::SortPairs(tmp, *tmp_bytes, kin, kout, vin, vout, (int)n, 0, (int)end_bit, st);
}

}  // namespace ks
