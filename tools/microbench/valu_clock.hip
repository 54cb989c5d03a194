// Microbenchmark: issue rate of the VALU instructions the verifier is built from, with the
// shader clock the chip actually held during the measurement, so that rates are stated per cycle instead of
// against the 2.4 GHz spec clock.
//
// Method (MI355X_MICROARCH.md "DVFS give-back" item 6): >= 2 s of back-to-back launches first; every wave stamps
// s_memtime (shader cycles) and s_memrealtime (100 MHz) around its loop; clock = median over waves of
// dcycles / dreal x 100 MHz.  8 waves per SIMD, 8 independent chains per lane (issue-bound, not latency-bound).
// Reported: lane-ops/s, the clock, and cycles per wave-instruction per SIMD at that clock.
//   v_fma_f32 same-src   the r01 form (src1 == src2: one VGPR read twice)
//   v_fma_f32            acc = a * b + acc, three distinct VGPRs
//   v_pk_fma_f32         two f32 lanes per instruction (VOP3P)
//   v_mad_u64_u32        the field multiply's product (32x32 -> 64 + 64)
//   v_add_u32 / v_lshl_add_u64 / v_mul_lo_u32 / v_bitop3_b32  the other classes of the comb step
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define ITERS 16384
#define CH 8

struct stamp { uint64_t c0, c1, r0, r1; };

#define BODY_BEGIN                                                      \
  uint64_t c0 = 0, r0 = 0;                                              \
  if ((threadIdx.x & 63) == 0) {                                        \
    r0 = __builtin_amdgcn_s_memrealtime();                              \
    c0 = __builtin_amdgcn_s_memtime();                                  \
  }
#define BODY_END(sink)                                                  \
  if ((threadIdx.x & 63) == 0) {                                        \
    const uint64_t c1 = __builtin_amdgcn_s_memtime();                   \
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();               \
    st[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = {c0, c1, r0, r1};\
  }                                                                     \
  out[blockIdx.x * blockDim.x + threadIdx.x] = (sink);

__global__ void k_fma_same(uint64_t* out, stamp* st, uint32_t seed) {
  float a = (float)(threadIdx.x + seed) * 1e-9f, acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  BODY_BEGIN
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(acc[c]) : "v"(a));
  float s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c];
  BODY_END((uint64_t)s)
}

__global__ void k_fma(uint64_t* out, stamp* st, uint32_t seed) {
  float a = (float)(threadIdx.x + seed) * 1e-9f, b = a * 0.5f + 1.0f, acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  BODY_BEGIN
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b));
  float s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c];
  BODY_END((uint64_t)s)
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
__global__ void k_pk_fma(uint64_t* out, stamp* st, uint32_t seed) {
  f32x2 a = {(float)(threadIdx.x + seed) * 1e-9f, 2.f}, b = {0.5f, 1.0f}, acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = a + (float)c;
  BODY_BEGIN
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b));
  float s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c].x + acc[c].y;
  BODY_END((uint64_t)s)
}

__global__ void k_mad64(uint64_t* out, stamp* st, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed, b = a ^ 0x9e3779b9u;
  uint64_t acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  BODY_BEGIN
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      uint64_t cc;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[c]), "=s"(cc) : "v"(a), "v"(b));
    }
  uint64_t s = 0;
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  BODY_END(s)
}

__global__ void k_add(uint64_t* out, stamp* st, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed, acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  BODY_BEGIN
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(acc[c]) : "v"(a));
  uint32_t s = 0;
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  BODY_END(s)
}

__global__ void k_lshl_add64(uint64_t* out, stamp* st, uint32_t seed) {
  uint64_t a = threadIdx.x * 2654435761ull + seed, acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  BODY_BEGIN
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[c]) : "v"(a));
  uint64_t s = 0;
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  BODY_END(s)
}

__global__ void k_mullo(uint64_t* out, stamp* st, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed, acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  BODY_BEGIN
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(a));
  uint32_t s = 0;
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  BODY_END(s)
}

__global__ void k_bitop3(uint64_t* out, stamp* st, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed, b = a * 3u, acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  BODY_BEGIN
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(acc[c]) : "v"(a), "v"(b));
  uint32_t s = 0;
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  BODY_END(s)
}


// generic 32-bit three-operand forms: acc = op(acc, a, b) with distinct VGPRs
#define K32(NAME, ASM)                                                                               \
  __global__ void NAME(uint64_t* out, stamp* st, uint32_t seed) {                                    \
    uint32_t a = threadIdx.x * 2654435761u + seed, b = a * 3u + 7u, acc[CH];                         \
    for (int c = 0; c < CH; ++c) acc[c] = a + c;                                                     \
    BODY_BEGIN                                                                                       \
    for (int i = 0; i < ITERS; ++i)                                                                  \
      _Pragma("unroll") for (int c = 0; c < CH; ++c) asm volatile(ASM : "+v"(acc[c]) : "v"(a), "v"(b) : "vcc", "s0", "s1"); \
    uint32_t s = 0;                                                                                  \
    for (int c = 0; c < CH; ++c) s ^= acc[c];                                                        \
    BODY_END(s)                                                                                      \
  }
K32(k_alignbit, "v_alignbit_b32 %0, %1, %0, 26")
K32(k_bfi, "v_bfi_b32 %0, %1, %0, %2")
K32(k_and, "v_and_b32_e32 %0, %1, %0")
K32(k_sub, "v_sub_u32_e32 %0, %1, %0")
K32(k_add3, "v_add3_u32 %0, %1, %0, %2")
K32(k_mul24, "v_mul_u32_u24_e32 %0, %1, %0")
K32(k_mad24, "v_mad_u32_u24 %0, %1, %0, %2")
K32(k_lshl_or, "v_lshl_or_b32 %0, %1, 6, %0")
K32(k_and_or, "v_and_or_b32 %0, %1, %2, %0")
K32(k_cndmask64, "v_cmp_lt_u32_e64 s[0:1], %1, %2\n v_cndmask_b32_e64 %0, %0, %1, s[0:1]")

// 64-bit shift: acc = acc >> 26 | a (kept live), the carry step's shift
__global__ void k_lshr64(uint64_t* out, stamp* st, uint32_t seed) {
  uint64_t a = threadIdx.x * 2654435761ull + seed, acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  BODY_BEGIN
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(acc[c]));
  uint64_t s = a;
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  BODY_END(s)
}

// 64-bit add as a VOP2 pair through VCC (v_add_co_u32 + v_addc_co_u32): counts 2 instructions per op
__global__ void k_addc_pair(uint64_t* out, stamp* st, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed, lo[CH], hi[CH];
  for (int c = 0; c < CH; ++c) { lo[c] = a + c; hi[c] = c; }
  BODY_BEGIN
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c)
      asm volatile("v_add_co_u32_e32 %0, vcc, %2, %0\n v_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
                   : "+v"(lo[c]), "+v"(hi[c]) : "v"(a) : "vcc");
  uint32_t s = 0;
  for (int c = 0; c < CH; ++c) s ^= lo[c] ^ hi[c];
  BODY_END(s)
}

typedef void (*kfn)(uint64_t*, stamp*, uint32_t);

int main() {
  const int blocks = 256 * 8, threads = 256;  // 8 waves per SIMD
  const int waves = blocks * threads / 64;
  uint64_t* d;
  stamp* dst;
  (void)hipMalloc(&d, sizeof(uint64_t) * blocks * threads);
  (void)hipMalloc(&dst, sizeof(stamp) * waves);
  std::vector<stamp> hs(waves);
  struct {
    const char* name;
    kfn f;
    int lanes_per_op;  // results per lane per instruction
  } ks[] = {{"v_fma_f32 same-src", k_fma_same, 1}, {"v_fma_f32", k_fma, 1}, {"v_pk_fma_f32", k_pk_fma, 2},
            {"v_mad_u64_u32", k_mad64, 1},     {"v_add_u32_e32", k_add, 1}, {"v_lshl_add_u64", k_lshl_add64, 1},
            {"v_mul_lo_u32", k_mullo, 1},      {"v_bitop3_b32", k_bitop3, 1},
            {"v_alignbit_b32", k_alignbit, 1}, {"v_bfi_b32", k_bfi, 1},   {"v_and_b32_e32", k_and, 1},
            {"v_sub_u32_e32", k_sub, 1},       {"v_add3_u32", k_add3, 1}, {"v_mul_u32_u24_e32", k_mul24, 1},
            {"v_mad_u32_u24", k_mad24, 1},     {"v_lshl_or_b32", k_lshl_or, 1}, {"v_and_or_b32", k_and_or, 1},
            {"v_cmp+v_cndmask_e64 (2)", k_cndmask64, 1}, {"v_lshrrev_b64", k_lshr64, 1},
            {"v_add_co+v_addc_co (2)", k_addc_pair, 1}};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  printf("%-20s %9s %10s %9s %12s %14s\n", "instruction", "ms", "T ops/s", "clock", "cyc/wave-ins", "@2.4GHz cyc");
  for (auto& k : ks) {
    // settle: >= 2 s of back-to-back launches (DVFS reaches its loaded clock)
    (void)hipEventRecord(e0);
    float warm = 0;
    while (warm < 2000.f) {
      for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, dst, 1u);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&warm, e0, e1);
    }
    float best = 1e30f;
    double clock = 0;
    for (int r = 0; r < 5; ++r) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, dst, (uint32_t)r);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) {
        best = ms;
        (void)hipMemcpy(hs.data(), dst, sizeof(stamp) * waves, hipMemcpyDeviceToHost);
        std::vector<double> f;
        for (auto& s : hs)
          if (s.r1 > s.r0) f.push_back((double)(s.c1 - s.c0) / (double)(s.r1 - s.r0) * 100e6);
        std::sort(f.begin(), f.end());
        clock = f.empty() ? 0 : f[f.size() / 2];
      }
    }
    const double wave_ins = (double)waves * ITERS * CH;        // wave-instructions
    const double ops = wave_ins * 64 * k.lanes_per_op;          // lane results
    const double simds = 256 * 4;
    const double cyc = best * 1e-3 * clock * simds / wave_ins;  // cycles per wave-instruction per SIMD
    const double cyc24 = best * 1e-3 * 2.4e9 * simds / wave_ins;
    printf("%-20s %9.3f %10.2f %7.3f G %12.2f %14.2f\n", k.name, best, ops / (best * 1e-3) / 1e12, clock / 1e9, cyc,
           cyc24);
  }
  return 0;
}
