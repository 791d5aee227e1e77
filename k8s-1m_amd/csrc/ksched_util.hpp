// ksched_util.hpp — device helpers shared by the round kernels
// (ksched_kernels.hip) and the in-order commit kernels (ksched_resolve.hip):
// wave reductions over DPP / readlane, kernel-side completion signals, round
// marks, the modified-slot hash and the resolve's node record.
#pragma once

#include <hip/hip_runtime.h>

#include <utility>

#include "ksched_dev.hpp"
#include "ksched_eval.hpp"

namespace ks {

constexpr int KS_PLUGIN_FIT_IDX = 4;  // filter status of NodeResourcesFit (KS_PLUGIN_FIT)
typedef __attribute__((address_space(1))) void gvoid_t;  // global_load_lds operands
typedef __attribute__((address_space(3))) void lvoid_t;

// Compile-time unrolled loop: keeps per-node register arrays statically indexed
// (a runtime-indexed array would be demoted to scratch).
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F &&f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    uint64_t o = __shfl_xor(v, m, WAVE);
    v = o > v ? o : v;
  }
  return v;
}

// Optimal 19-comparator network, descending (static indices only).
__device__ __forceinline__ void cx_desc(uint64_t &a, uint64_t &b) {
  const uint64_t hi = a > b ? a : b, lo = a > b ? b : a;
  a = hi;
  b = lo;
}
__device__ __forceinline__ void sort8_desc(uint64_t *k) {
  cx_desc(k[0], k[2]); cx_desc(k[1], k[3]); cx_desc(k[4], k[6]); cx_desc(k[5], k[7]);
  cx_desc(k[0], k[4]); cx_desc(k[1], k[5]); cx_desc(k[2], k[6]); cx_desc(k[3], k[7]);
  cx_desc(k[0], k[1]); cx_desc(k[2], k[3]); cx_desc(k[4], k[5]); cx_desc(k[6], k[7]);
  cx_desc(k[2], k[4]); cx_desc(k[3], k[5]);
  cx_desc(k[1], k[4]); cx_desc(k[3], k[6]);
  cx_desc(k[1], k[2]); cx_desc(k[3], k[4]); cx_desc(k[5], k[6]);
}

// the builtin takes the compare's lane mask as is (__ballot(int) made the
// compiler copy it into a VGPR and compare it again)
__device__ __forceinline__ uint32_t popc_ballot(bool b) {
  return (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(b));
}

// v where the lane's bit of the wave mask m is set, else 0
__device__ __forceinline__ uint32_t sel_mask(uint64_t m, uint32_t v) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(r) : "v"(v), "s"(m));
  return r;
}

__device__ __forceinline__ uint32_t uniform_u32(uint32_t v) {
  return __builtin_amdgcn_readfirstlane(v);
}

// max of two wave-uniform values on the SALU (left to itself the compiler
// moves the row maxima into VGPRs for one v_max3: three VALU per reduction)
__device__ __forceinline__ uint32_t smax_u32(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("s_max_u32 %0, %1, %2" : "=s"(r) : "s"(a), "s"(b) : "scc");
  return r;
}

// DPP lane moves (no LDS): quad_perm(1,0,3,2) = 0xB1, quad_perm(2,3,0,1) = 0x4E,
// row_half_mirror = 0x141, row_mirror = 0x140.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  return ((uint64_t)dpp32<CTRL>((uint32_t)(v >> 32)) << 32) | dpp32<CTRL>((uint32_t)v);
}
__device__ __forceinline__ uint64_t max64(uint64_t a, uint64_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}
// max over each 8-lane group (every lane of the group holds it)
__device__ __forceinline__ uint64_t max8_u64(uint64_t v) {
  v = max64(v, dpp64<0xB1>(v));
  v = max64(v, dpp64<0x4E>(v));
  return max64(v, dpp64<0x141>(v));
}
// wave max, wave-uniform result
__device__ __forceinline__ uint64_t wave_max_u64_dpp(uint64_t v) {
  v = max8_u64(v);
  v = max64(v, dpp64<0x140>(v));
  return max64(max64(readlane64(v, 0), readlane64(v, 16)), max64(readlane64(v, 32), readlane64(v, 48)));
}
__device__ __forceinline__ uint32_t wave_max_u32_dpp(uint32_t v) {
  v = max(v, dpp32<0xB1>(v));
  v = max(v, dpp32<0x4E>(v));
  v = max(v, dpp32<0x141>(v));
  v = max(v, dpp32<0x140>(v));
  return smax_u32(smax_u32((uint32_t)__builtin_amdgcn_readlane((int)v, 0), (uint32_t)__builtin_amdgcn_readlane((int)v, 16)),
                  smax_u32((uint32_t)__builtin_amdgcn_readlane((int)v, 32), (uint32_t)__builtin_amdgcn_readlane((int)v, 48)));
}
__device__ __forceinline__ uint32_t min8_u32(uint32_t v) {
  v = min(v, dpp32<0xB1>(v));
  v = min(v, dpp32<0x4E>(v));
  return min(v, dpp32<0x141>(v));
}
__device__ __forceinline__ int32_t sum8_i32(int32_t v) {
  v += (int32_t)dpp32<0xB1>((uint32_t)v);
  v += (int32_t)dpp32<0x4E>((uint32_t)v);
  return v + (int32_t)dpp32<0x141>((uint32_t)v);
}
__device__ __forceinline__ int32_t wave_sum_i32_dpp(int32_t v) {
  v = sum8_i32(v);
  v += (int32_t)dpp32<0x140>((uint32_t)v);
  return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
         __builtin_amdgcn_readlane(v, 48);
}

// Bounded wall-clock wait (ks_debug_stall): s_memrealtime counts at 100 MHz.
__device__ __forceinline__ void stall_for(uint32_t usec) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < 100ull * usec) __builtin_amdgcn_s_sleep(127);
}

// Kernel-side completion signal for a stream wait-value (release at system
// scope, like the stream write operation it replaces).
__device__ __forceinline__ void signal_done(uint32_t *flag, uint32_t seq, uint32_t stall_us = 0) {
  if (flag == nullptr) return;
  if (stall_us) stall_for(stall_us);
  __threadfence_system();
  __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Round marks (diagnostics, ks_batch_marks): byte i of a word-aligned
// buffer, set atomically (the main stream's norm_check and the resolve stream
// may mark pods of one word concurrently).
__device__ __forceinline__ void mark_pod(uint8_t *marks, uint32_t i, uint8_t bit) {
  atomicOr((uint32_t *)(marks + (i & ~3u)), (uint32_t)bit << (8u * (i & 3u)));
}

__device__ __forceinline__ uint32_t rhash(uint32_t x) { return (x * 2654435761u) >> 22; }  // 10 bits

// A node as the resolve carries it: its row (live state) and the round-start
// Requested / pod count its listed key was computed from.
struct alignas(16) RNode {
  CandRow row;       // live
  double rc0, rm0;   // Requested at the round start
  int32_t np0;
  uint32_t slot;
  uint32_t _pad[2];
};
static_assert(sizeof(RNode) == 112, "RNode layout");

__device__ __forceinline__ RNode rnode_from_row(const CandRow &w, uint32_t slot) {
  RNode n;
  n.row = w;
  n.rc0 = w.rc;
  n.rm0 = w.rm;
  n.np0 = w.np;
  n.slot = slot;
  n._pad[0] = n._pad[1] = 0;
  return n;
}

// NodeInfo.AddPod on the live state (AssumePod): exact binary64 additions
__device__ __forceinline__ void rnode_add(RNode &n, const PodDev &p) {
  n.row.rc += p.req_cpu_d;
  n.row.rm += p.req_mem_d;
  n.row.zc100 += p.nz100_cpu;
  n.row.zm100 += p.nz100_mem;
  n.row.np += 1;
}

// NodeRegs of the node with Requested (rc, rm) and pod count np: no int64 ->
// binary64 conversion, every value exact (allocatable < 2^44).
__device__ __forceinline__ NodeRegs rnode_regs(const RNode &n, double rc, double rm, int32_t np) {
  const CandRow &w = n.row;
  NodeRegs r;
  r.slot = n.slot;
  r.free_cpu = w.acpu - rc;
  r.free_mem = w.amem - rm;
  r.rcpu = rc;
  r.rmem = rm;
  r.lf100_cpu = w.acpu * 100.0 - w.zc100;
  r.lf100_mem = w.amem * 100.0 - w.zm100;
  r.acpu_d = w.acpu;
  r.amem_d = w.amem;
  r.inv_cpu = w.inv_cpu;
  r.inv_mem = w.inv_mem;
  const bool ac = w.acpu != 0.0, am = w.amem != 0.0;
  r.bamul = (ac && am) ? 0.5 : 0.0;
  r.lashift = (ac && am) ? 1u : 0u;
  r.bits = 1u | (np + 1 <= w.apods ? 2u : 0u) | (ac ? 4u : 0u) | (am ? 8u : 0u);
  return r;
}

// Carry record (the next round's patch and the write-back) of a modified node.
__device__ __forceinline__ CarryRec rnode_carry(const RNode &n, const CandExt &x, bool ext) {
  const CandRow &w = n.row;
  CarryRec c;
  c.acpu = (int64_t)w.acpu;
  c.amem = (int64_t)w.amem;
  c.rc0 = (int64_t)n.rc0;
  c.rm0 = (int64_t)n.rm0;
  c.np0 = n.np0;
  c.rc = (int64_t)w.rc;
  c.rm = (int64_t)w.rm;
  c.zc = (int64_t)(w.zc100 / 100.0);  // exact: zc100 is 100 zc
  c.zm = (int64_t)(w.zm100 / 100.0);
  c.np = w.np;
  c.slot = n.slot;
  c.pos = w.pos;
  c.apods = w.apods;
  c._pad = 0;
#pragma unroll
  for (int q = 0; q < 2 + LW + NNUM; ++q) c.ext[q] = ext ? x.w[q] : 0ull;
  return c;
}

// Workgroup barrier for LDS hand-offs only: __syncthreads() also drains vmcnt,
// which would drain the list waves' LDS-DMA pipeline on every iteration.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

}  // namespace ks
