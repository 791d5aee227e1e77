// valu_issue.hip -- issue cost of the VALU instructions the sweep kernel is
// made of, on gfx950 (MI355X), at 1, 2 and 4 waves per SIMD.
//
// Each kernel runs one block of W x 256 threads (W waves per SIMD) per CU;
// every wave issues ITERS x 32 copies of one instruction on 8 independent
// register chains (so dependency latency hides behind the other chains and
// waves), timing itself with s_memtime (shader clock cycles).  With W waves
// sharing a SIMD, the issue cost of one wave64 instruction is
//     cycles per wave / (instructions per wave x W).
// Output: one JSON object per line {instr, waves_per_simd, cycles_per_instr,
// clock_ghz}; bench.py reads profiles/valu_issue.json to price the sweep's
// measured instruction mix.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/valu_issue tools/valu_issue.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                              \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      std::fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                               \
    }                                                                                         \
  } while (0)

constexpr int ITERS = 8192;  // ~1 ms per launch: start skew and launch overhead negligible
constexpr int PER_ITER = 32;  // 4 x 8 chains

#define REP4(X) X X X X

// per wave: start / end shader cycle, real-time ticks (100 MHz) and the
// hardware id (HW_REG_HW_ID: SIMD in bits 5:4), 4 words at (block * 16 + wave) * 4
__device__ __forceinline__ void record(unsigned long long *cyc, unsigned long long t0, unsigned long long t1,
                                       unsigned long long r0, unsigned long long r1) {
  unsigned long long *o = cyc + ((size_t)blockIdx.x * 16 + threadIdx.x / 64) * 4;
  o[0] = t0;
  o[1] = t1;
  o[2] = r1 - r0;
  o[3] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
}

// 64-bit accumulators (f64 / b64 ops)
#define K64(NAME, INSTR)                                                                                      \
  __global__ void NAME(unsigned long long *cyc, double seed, double c, uint32_t iters) {                       \
    double a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3, a4 = seed + 4, a5 = seed + 5, a6 = seed + 6, \
           a7 = seed + 7;                                                                                      \
    const unsigned long long t0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();       \
    for (uint32_t i = 0; i < iters; ++i) {                                                                    \
      asm volatile(REP4(INSTR(0) INSTR(1) INSTR(2) INSTR(3) INSTR(4) INSTR(5) INSTR(6) INSTR(7))              \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)           \
                   : "v"(c)                                                                                    \
                   : "vcc", "s0", "s1");                                                                                   \
    }                                                                                                          \
    const unsigned long long t1 = __builtin_readcyclecounter(), r1 = __builtin_amdgcn_s_memrealtime();       \
    if (threadIdx.x % 64 == 0) record(cyc, t0, t1, r0, r1);        \
    if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 1.2345) cyc[0] = 0;                                          \
  }

// 32-bit accumulators
#define K32(NAME, INSTR)                                                                                        \
  __global__ void NAME(unsigned long long *cyc, uint32_t seed, uint32_t c, uint32_t iters) {                    \
    uint32_t a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3, a4 = seed + 4, a5 = seed + 5, a6 = seed + 6, \
             a7 = seed + 7;                                                                                     \
    const double dc = (double)c;                                                                                \
    const uint32_t c2 = c + 1u + (threadIdx.x & 1u); /* a second VGPR source */                                 \
    const unsigned long long m = __builtin_amdgcn_read_exec() & 0x5555555555555555ull;                         \
    const unsigned long long t0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();        \
    for (uint32_t i = 0; i < iters; ++i) {                                                                     \
      asm volatile(REP4(INSTR(0) INSTR(1) INSTR(2) INSTR(3) INSTR(4) INSTR(5) INSTR(6) INSTR(7))               \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)            \
                   : "v"(c), "s"(m), "v"(dc), "v"(c2), "s"(c)                                                  \
                   : "vcc", "s0", "s1");                                                                                    \
    }                                                                                                           \
    const unsigned long long t1 = __builtin_readcyclecounter(), r1 = __builtin_amdgcn_s_memrealtime();        \
    if (threadIdx.x % 64 == 0) record(cyc, t0, t1, r0, r1);         \
    if ((a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) == 0x12345u) cyc[0] = 0;                                       \
  }

// operand %8: c (32-bit: v, 64-bit: v pair); %9: SGPR mask; %10: c as double;
// 32-bit only: %11 a second VGPR (c2), %12 c in an SGPR.  The f32 FMA
// variants separate the opcode from the encoding and the operand sources:
// v_fma_f32 is VOP3-only; v_fmac_f32 is its VOP2 form (the destination is the
// addend); the _e64 adds are VOP2 opcodes forced into the VOP3 encoding.
#define I_ADD_F64(r) "v_add_f64 %" #r ", %" #r ", %8\n"
#define I_MUL_F64(r) "v_mul_f64 %" #r ", %" #r ", %8\n"
#define I_FMA_F64(r) "v_fma_f64 %" #r ", %" #r ", %8, %8\n"
#define I_LSHL_B64(r) "v_lshlrev_b64 %" #r ", 1, %" #r "\n"
#define I_CMP_F64(r) "v_cmp_gt_f64 vcc, %" #r ", %8\n"
#define I_ADD_U32(r) "v_add_u32 %" #r ", %" #r ", %8\n"
#define I_FMA_F32(r) "v_fma_f32 %" #r ", %" #r ", %8, %8\n"
#define I_MUL_U24(r) "v_mul_u32_u24 %" #r ", %" #r ", %8\n"
#define I_MAD_U24(r) "v_mad_u32_u24 %" #r ", %" #r ", %8, %8\n"
#define I_MUL_LO(r) "v_mul_lo_u32 %" #r ", %" #r ", %8\n"
#define I_CNDMASK(r) "v_cndmask_b32 %" #r ", %" #r ", %8, %9\n"
#define I_DPP(r) "v_mov_b32_dpp %" #r ", %8 row_shr:1 row_mask:0xf bank_mask:0xf\n"
#define I_CVT_U32_F64(r) "v_cvt_u32_f64 %" #r ", %10\n"
#define I_AND(r) "v_and_b32 %" #r ", %" #r ", %8\n"
#define I_MAX3(r) "v_max3_u32 %" #r ", %" #r ", %8, %8\n"
#define I_FMAC_F64(r) "v_fmac_f64 %" #r ", %8, %8\n"
#define I_MIN_F64(r) "v_min_f64 %" #r ", %" #r ", %8\n"
#define I_MOV_B64(r) "v_mov_b64 %" #r ", %8\n"
#define I_CMP_U64(r) "v_cmp_lt_u64 vcc, %" #r ", %8\n"
#define I_MAD_U64(r) "v_mad_u64_u32 %" #r ", s[0:1], %8, %8, %" #r "\n"
#define I_CVT_I32_F64(r) "v_cvt_i32_f64 %" #r ", %10\n"
#define I_MAXU_DPP(r) "v_max_u32_dpp %" #r ", %8, %" #r " row_shr:1 row_mask:0xf bank_mask:0xf\n"
#define I_MOV_B32(r) "v_mov_b32 %" #r ", %8\n"
#define I_ASHR(r) "v_ashrrev_i32 %" #r ", 3, %" #r "\n"
#define I_NOT(r) "v_not_b32 %" #r ", %" #r "\n"
#define I_MINU(r) "v_min_u32 %" #r ", %" #r ", %8\n"
#define I_MAXU(r) "v_max_u32 %" #r ", %" #r ", %8\n"
#define I_CND_VCC(r) "v_cndmask_b32 %" #r ", %" #r ", %8, vcc\n"
#define I_CMP_NE(r) "v_cmp_ne_u32 vcc, %" #r ", %8\n"
#define I_XOR(r) "v_xor_b32 %" #r ", %" #r ", %8\n"
#define I_LSHL(r) "v_lshlrev_b32 %" #r ", 1, %" #r "\n"
#define I_ADD_F32(r) "v_add_f32 %" #r ", %" #r ", %8\n"
#define I_MUL_F32(r) "v_mul_f32 %" #r ", %" #r ", %8\n"
#define I_SUB_U32(r) "v_sub_u32 %" #r ", %" #r ", %8\n"
#define I_ADD3(r) "v_add3_u32 %" #r ", %" #r ", %8, %8\n"
#define I_BFE(r) "v_bfe_u32 %" #r ", %" #r ", 3, 5\n"
#define I_FMA_F32_2V(r) "v_fma_f32 %" #r ", %" #r ", %8, %11\n"
#define I_FMA_F32_SV(r) "v_fma_f32 %" #r ", %" #r ", %12, %8\n"
#define I_FMAC_F32(r) "v_fmac_f32 %" #r ", %8, %11\n"
#define I_FMAC_F32_SAME(r) "v_fmac_f32 %" #r ", %8, %8\n"
#define I_ADD_F32_E64(r) "v_add_f32_e64 %" #r ", %" #r ", %8\n"
#define I_MUL_F32_E64(r) "v_mul_f32_e64 %" #r ", %" #r ", %8\n"
#define I_ADD_U32_E64(r) "v_add_u32_e64 %" #r ", %" #r ", %8\n"
// an SGPR source (src0) in the 2-cycle class
#define I_ADD_F32_S(r) "v_add_f32 %" #r ", %12, %" #r "\n"
#define I_MUL_F32_S(r) "v_mul_f32 %" #r ", %12, %" #r "\n"
#define I_ADD_U32_S(r) "v_add_u32 %" #r ", %12, %" #r "\n"
#define I_AND_S(r) "v_and_b32 %" #r ", %12, %" #r "\n"
#define I_FMAC_F32_S(r) "v_fmac_f32 %" #r ", %12, %8\n"
#define I_FMA_F32_SS(r) "v_fma_f32 %" #r ", %12, %12, %" #r "\n"

K64(k_add_f64, I_ADD_F64)
K64(k_mul_f64, I_MUL_F64)
K64(k_fma_f64, I_FMA_F64)
K64(k_lshl_b64, I_LSHL_B64)
K64(k_cmp_f64, I_CMP_F64)
K32(k_add_u32, I_ADD_U32)
K32(k_fma_f32, I_FMA_F32)
K32(k_mul_u24, I_MUL_U24)
K32(k_mad_u24, I_MAD_U24)
K32(k_mul_lo_u32, I_MUL_LO)
K32(k_cndmask, I_CNDMASK)
K32(k_dpp_mov, I_DPP)
K32(k_cvt_u32_f64, I_CVT_U32_F64)
K32(k_and_b32, I_AND)
K32(k_max3_u32, I_MAX3)
K64(k_fmac_f64, I_FMAC_F64)
K64(k_min_f64, I_MIN_F64)
K64(k_mov_b64, I_MOV_B64)
K64(k_cmp_u64, I_CMP_U64)
K32(k_cvt_i32_f64, I_CVT_I32_F64)
K32(k_maxu_dpp, I_MAXU_DPP)
K32(k_mov_b32, I_MOV_B32)
K32(k_ashr, I_ASHR)
K32(k_not, I_NOT)
K32(k_minu, I_MINU)
K32(k_maxu, I_MAXU)
K32(k_cnd_vcc, I_CND_VCC)
K32(k_cmp_ne, I_CMP_NE)
K32(k_xor, I_XOR)
K32(k_lshl, I_LSHL)
K32(k_add_f32, I_ADD_F32)
K32(k_mul_f32, I_MUL_F32)
K32(k_sub_u32, I_SUB_U32)
K32(k_add3, I_ADD3)
K32(k_bfe, I_BFE)
K32(k_fma_f32_2v, I_FMA_F32_2V)
K32(k_fma_f32_sv, I_FMA_F32_SV)
K32(k_fmac_f32, I_FMAC_F32)
K32(k_fmac_f32_same, I_FMAC_F32_SAME)
K32(k_add_f32_e64, I_ADD_F32_E64)
K32(k_mul_f32_e64, I_MUL_F32_E64)
K32(k_add_u32_e64, I_ADD_U32_E64)
K32(k_add_f32_s, I_ADD_F32_S)
K32(k_mul_f32_s, I_MUL_F32_S)
K32(k_add_u32_s, I_ADD_U32_S)
K32(k_and_s, I_AND_S)
K32(k_fmac_f32_s, I_FMAC_F32_S)
K32(k_fma_f32_ss, I_FMA_F32_SS)

// v_readlane_b32: SGPR destinations
__global__ void k_readlane(unsigned long long *cyc, uint32_t seed, uint32_t c, uint32_t iters) {
  uint32_t v = seed + threadIdx.x, s0, s1, s2, s3, s4, s5, s6, s7;
  const unsigned long long t0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t i = 0; i < iters; ++i) {
#define I_RL(r) "v_readlane_b32 %" #r ", %8, 5\n"
    asm volatile(REP4(I_RL(0) I_RL(1) I_RL(2) I_RL(3) I_RL(4) I_RL(5) I_RL(6) I_RL(7))
                 : "=s"(s0), "=s"(s1), "=s"(s2), "=s"(s3), "=s"(s4), "=s"(s5), "=s"(s6), "=s"(s7)
                 : "v"(v));
  }
  const unsigned long long t1 = __builtin_readcyclecounter(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x % 64 == 0) record(cyc, t0, t1, r0, r1);
  if ((s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7) == 0x12345u) cyc[0] = c;
}

// v_cvt_f64_u32: 64-bit destinations from a 32-bit source
__global__ void k_cvt_f64_u32(unsigned long long *cyc, double seed, double c, uint32_t iters) {
  double a0 = seed, a1 = seed, a2 = seed, a3 = seed, a4 = seed, a5 = seed, a6 = seed, a7 = seed;
  const uint32_t src = (uint32_t)c + threadIdx.x;
  const unsigned long long t0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t i = 0; i < iters; ++i) {
#define I_CVT_F64_U32(r) "v_cvt_f64_u32 %" #r ", %8\n"
    asm volatile(REP4(I_CVT_F64_U32(0) I_CVT_F64_U32(1) I_CVT_F64_U32(2) I_CVT_F64_U32(3) I_CVT_F64_U32(4)
                          I_CVT_F64_U32(5) I_CVT_F64_U32(6) I_CVT_F64_U32(7))
                 : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7)
                 : "v"(src));
  }
  const unsigned long long t1 = __builtin_readcyclecounter(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x % 64 == 0) record(cyc, t0, t1, r0, r1);
  if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 1.2345) cyc[0] = 0;
}

using K64F = void (*)(unsigned long long *, double, double, uint32_t);
using K32F = void (*)(unsigned long long *, uint32_t, uint32_t, uint32_t);

struct Entry {
  const char *name;
  K64F k64;
  K32F k32;
};

int main() {
  const Entry tab[] = {
      {"v_add_f64", k_add_f64, nullptr},         {"v_mul_f64", k_mul_f64, nullptr},
      {"v_fma_f64", k_fma_f64, nullptr},         {"v_lshlrev_b64", k_lshl_b64, nullptr},
      {"v_cmp_gt_f64", k_cmp_f64, nullptr},      {"v_cvt_f64_u32", k_cvt_f64_u32, nullptr},
      {"v_cvt_u32_f64", nullptr, k_cvt_u32_f64}, {"v_add_u32", nullptr, k_add_u32},
      {"v_fma_f32", nullptr, k_fma_f32},         {"v_mul_u32_u24", nullptr, k_mul_u24},
      {"v_mad_u32_u24", nullptr, k_mad_u24},     {"v_mul_lo_u32", nullptr, k_mul_lo_u32},
      {"v_cndmask_b32", nullptr, k_cndmask},     {"v_mov_b32_dpp", nullptr, k_dpp_mov},
      {"v_and_b32", nullptr, k_and_b32},         {"v_max3_u32", nullptr, k_max3_u32},
      {"v_fmac_f64", k_fmac_f64, nullptr},       {"v_min_f64", k_min_f64, nullptr},
      {"v_mov_b64", k_mov_b64, nullptr},         {"v_cmp_lt_u64", k_cmp_u64, nullptr},
      {"v_cvt_i32_f64", nullptr, k_cvt_i32_f64}, {"v_max_u32_dpp", nullptr, k_maxu_dpp},
      {"v_mov_b32", nullptr, k_mov_b32},         {"v_ashrrev_i32", nullptr, k_ashr},
      {"v_not_b32", nullptr, k_not},             {"v_min_u32", nullptr, k_minu},
      {"v_max_u32", nullptr, k_maxu},            {"v_cndmask_b32_vcc", nullptr, k_cnd_vcc},
      {"v_cmp_ne_u32", nullptr, k_cmp_ne},       {"v_xor_b32", nullptr, k_xor},
      {"v_lshlrev_b32", nullptr, k_lshl},        {"v_add_f32", nullptr, k_add_f32},
      {"v_mul_f32", nullptr, k_mul_f32},         {"v_sub_u32", nullptr, k_sub_u32},
      {"v_add3_u32", nullptr, k_add3},           {"v_bfe_u32", nullptr, k_bfe},
      {"v_readlane_b32", nullptr, k_readlane},
      // VOP2 vs VOP3 (profiles/valu_vop.jsonl)
      {"v_fma_f32 (v, v', same v twice)", nullptr, k_fma_f32},
      {"v_fma_f32 (v, v', v'')", nullptr, k_fma_f32_2v},
      {"v_fma_f32 (v, s, v')", nullptr, k_fma_f32_sv},
      {"v_fmac_f32 (VOP2, v', v'')", nullptr, k_fmac_f32},
      {"v_fmac_f32 (VOP2, same v twice)", nullptr, k_fmac_f32_same},
      {"v_add_f32_e64 (VOP3)", nullptr, k_add_f32_e64},
      {"v_mul_f32_e64 (VOP3)", nullptr, k_mul_f32_e64},
      {"v_add_u32_e64 (VOP3)", nullptr, k_add_u32_e64},
      // an SGPR source operand
      {"v_add_f32 (s, v)", nullptr, k_add_f32_s},
      {"v_mul_f32 (s, v)", nullptr, k_mul_f32_s},
      {"v_add_u32 (s, v)", nullptr, k_add_u32_s},
      {"v_and_b32 (s, v)", nullptr, k_and_s},
      {"v_fmac_f32 (VOP2, s, v')", nullptr, k_fmac_f32_s},
      {"v_fma_f32 (s, s, v)", nullptr, k_fma_f32_ss},
  };
  const char *only = std::getenv("VALU_ONLY");  // a substring: run the matching entries only
  hipDeviceProp_t prop{};
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  unsigned long long *d = nullptr;
  CHECK(hipMalloc(&d, (size_t)ncu * 16 * 4 * sizeof(unsigned long long)));
  std::vector<unsigned long long> h((size_t)ncu * 16 * 4);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (const Entry &t : tab) {
    if (only && !std::strstr(t.name, only)) continue;
    for (int w : {1, 2, 4}) {
      const dim3 grid(ncu), block(256 * w);
      for (int rep = 0; rep < 2; ++rep) {  // first launch warms the clocks / caches
        CHECK(hipMemset(d, 0, h.size() * sizeof(unsigned long long)));
        CHECK(hipEventRecord(e0));
        if (t.k64) hipLaunchKernelGGL(t.k64, grid, block, 0, 0, d, 1.0000001, 1.0000003, (uint32_t)ITERS);
        else hipLaunchKernelGGL(t.k32, grid, block, 0, 0, d, 3u, 5u, (uint32_t)ITERS);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
      }
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      CHECK(hipMemcpy(h.data(), d, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      // per (CU, SIMD): the span from its first wave's start to its last
      // wave's end, over the instructions its waves issued
      std::vector<double> cost;
      std::vector<int> nw;
      double ghz_sum = 0;
      int ghz_n = 0;
      for (int b = 0; b < ncu; ++b) {
        for (int simd = 0; simd < 4; ++simd) {
          unsigned long long lo = ~0ull, hi = 0;
          int n = 0;
          for (int q = 0; q < 4 * w; ++q) {
            const unsigned long long *o = &h[((size_t)b * 16 + q) * 4];
            if (((o[3] >> 4) & 3) != (unsigned long long)simd) continue;
            lo = std::min(lo, o[0]);
            hi = std::max(hi, o[1]);
            ++n;
            if (o[2]) {
              ghz_sum += (double)(o[1] - o[0]) / ((double)o[2] * 10.0);
              ++ghz_n;
            }
          }
          if (n) {
            cost.push_back((double)(hi - lo) / ((double)ITERS * PER_ITER * n));
            nw.push_back(n);
          }
        }
      }
      std::sort(cost.begin(), cost.end());
      std::sort(nw.begin(), nw.end());
      std::printf("{\"instr\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_instr\": %.3f, \"p10\": %.3f, "
                  "\"p90\": %.3f, \"waves_per_simd_min\": %d, \"waves_per_simd_max\": %d, \"clock_ghz\": %.3f, "
                  "\"launch_ms\": %.3f}\n",
                  t.name, w, cost[cost.size() / 2], cost[cost.size() / 10], cost[cost.size() * 9 / 10], nw.front(),
                  nw.back(), ghz_sum / std::max(1, ghz_n), ms);
    }
  }
  CHECK(hipFree(d));
  return 0;
}
