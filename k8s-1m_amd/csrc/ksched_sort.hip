// ksched_sort.hip — device radix sort of (64-bit key, 64-bit value) pairs
// (rocPRIM onesweep), kept in its own translation unit: the replica runs of
// the spread path (ksched_spread.hip) order a run's feasible
// nodes by (group, static score descending) once per run, carrying each
// node's position; the keys sit at their slots, so equal keys stay in slot
// order.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include "ksched_kernels.hpp"

namespace ks {

// rocPRIM sorts up to 2^20 items by merge sort by default (10 merge passes of
// two kernels for a 1M-slot table, ~190 us); a merge-sort limit of 0 selects
// the onesweep LSD radix passes over the key's end_bit bits (stable).
using OnesweepOnly =
    rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;

// tmp == nullptr: *tmp_bytes = the scratch a sort of n pairs needs.
// Stable: equal keys keep their input order.  Bits [0, end_bit) are sorted.
hipError_t launch_sort_pairs(const uint64_t *kin, uint64_t *kout, const uint64_t *vin, uint64_t *vout, uint32_t n,
                             uint32_t end_bit, void *tmp, size_t *tmp_bytes, hipStream_t st) {
  return rocprim::radix_sort_pairs<OnesweepOnly>(tmp, *tmp_bytes, kin, kout, vin, vout, n, 0u, end_bit, st);
}

}  // namespace ks
