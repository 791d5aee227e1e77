// ksched_instr.hpp — instrumentation hooks of the serial resolve kernel
// (ksched_resolve_serial.hpp resolve_serial).  The product library is built without
// any of the switches below and every hook expands to nothing; only the
// diagnostic variants of k8s-1m_amd/Makefile define them:
//
//   KS_STAMPS=1..4  (make stamps / stamps2 / stamps3 / stamps4): one lane of
//       one wave accumulates s_memtime of its work and barrier wait per pod,
//       and of up to four sub-phases of its role (1 decider, 2 eval wave,
//       3 owner wave 0, 4 list wave 0), into the debug counters [8..15]
//       (tools/resolve_stamps.py reads them).  Never measured as the product.
//   KS_RACE_PROBE   (make probe): every wave but the decider reads the done
//       word late in the last two iterations, so the decider's next store
//       lands first (the regression case of tests/test_gpu_stall.py for the
//       double-buffered exit flag).
#pragma once

#ifdef KS_STAMPS
#define KS_STAMP_NOW(t_)                                                      \
  do {                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                        \
  } while (0)
// per-kernel state: which lane stamps, into which counters
#define KS_STAMP_DECL(wid_, lane_)                                                                         \
  const bool ks_stamper = (lane_) == 0 && (KS_STAMPS >= 3 ? ((wid_) == 0 || (wid_) == RES_LIST_WAVES)      \
                                                          : ((wid_) == RES_DEC_WAVE || (wid_) == RES_EVAL_WAVE)); \
  const uint32_t ks_sidx = KS_STAMPS >= 3 ? ((wid_) == 0 ? 0u : 2u) : ((wid_) == RES_DEC_WAVE ? 0u : 2u); \
  uint64_t ks_work = 0, ks_wait = 0, ks_t0 = 0, ks_t1 = 0, ks_t2 = 0, ks_ts = 0, ks_sub[4] = {0, 0, 0, 0}
// start of one pod's iteration
#define KS_STAMP_BEGIN() \
  do {                   \
    KS_STAMP_NOW(ks_t0); \
    ks_t2 = ks_t0;       \
  } while (0)
// end of sub-phase i_ of the role stamped by build level lvl_ (LGKM: after
// the phase's LDS loads have landed)
#define KS_STAMP_SPLIT(lvl_, i_)  \
  do {                            \
    if (KS_STAMPS == (lvl_)) {    \
      KS_STAMP_NOW(ks_ts);        \
      ks_sub[i_] += ks_ts - ks_t2; \
      ks_t2 = ks_ts;              \
    }                             \
  } while (0)
#define KS_STAMP_SPLIT_LGKM(lvl_, i_)                        \
  do {                                                       \
    if (KS_STAMPS == (lvl_)) {                               \
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     \
      KS_STAMP_SPLIT(lvl_, i_);                              \
    }                                                        \
  } while (0)
// around the per-pod barrier
#define KS_STAMP_PRE_BARRIER() KS_STAMP_NOW(ks_t1)
#define KS_STAMP_POST_BARRIER() \
  do {                          \
    KS_STAMP_NOW(ks_t2);        \
    ks_work += ks_t1 - ks_t0;   \
    ks_wait += ks_t2 - ks_t1;   \
  } while (0)
// after the loop: into the debug counters (vector global atomics)
#define KS_STAMP_FLUSH(counters_, wid_)                                                                       \
  do {                                                                                                        \
    if (ks_stamper) {                                                                                         \
      atomicAdd((unsigned long long *)&(counters_)[8 + ks_sidx], (unsigned long long)ks_work);                \
      atomicAdd((unsigned long long *)&(counters_)[9 + ks_sidx], (unsigned long long)ks_wait);                \
      const uint32_t ks_subw = KS_STAMPS == 4   ? 0u                                                          \
                               : KS_STAMPS == 3 ? (uint32_t)RES_LIST_WAVES                                    \
                               : KS_STAMPS == 2 ? (uint32_t)RES_EVAL_WAVE                                     \
                                                : (uint32_t)RES_DEC_WAVE;                                     \
      if ((wid_) == ks_subw)                                                                                  \
        for (int i = 0; i < 4; ++i) atomicAdd((unsigned long long *)&(counters_)[12 + i], (unsigned long long)ks_sub[i]); \
    }                                                                                                         \
  } while (0)
#else
#define KS_STAMP_DECL(wid_, lane_) static_assert(true, "")
#define KS_STAMP_BEGIN() ((void)0)
#define KS_STAMP_SPLIT(lvl_, i_) ((void)0)
#define KS_STAMP_SPLIT_LGKM(lvl_, i_) ((void)0)
#define KS_STAMP_PRE_BARRIER() ((void)0)
#define KS_STAMP_POST_BARRIER() ((void)0)
#define KS_STAMP_FLUSH(counters_, wid_) ((void)0)
#endif

#ifdef KS_RACE_PROBE
#define KS_RACE_DELAY(cond_)                                        \
  do {                                                              \
    if (cond_)                                                      \
      for (int ks_i = 0; ks_i < 8; ++ks_i) __builtin_amdgcn_s_sleep(127); \
  } while (0)
#else
#define KS_RACE_DELAY(cond_) ((void)0)
#endif
