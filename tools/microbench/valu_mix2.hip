// Which VOP2/VOP3 integer ops issue at the fast (~2.2 cycles per wave64) rate on gfx950, and whether a
// literal or SGPR operand changes it.  Same harness as valu_mix.hip: 8 independent chains per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 16384
#define CH 8
#define K32(name, body)                                                                              \
  __global__ void name(uint64_t* out, uint32_t seed) {                                               \
    uint32_t a = threadIdx.x * 2654435761u + seed;                                                   \
    uint32_t b = __builtin_amdgcn_readfirstlane(seed * 77u + 5u);                                    \
    uint32_t acc[CH];                                                                                \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) acc[c] = a + c;                                   \
    for (int i = 0; i < ITERS; ++i) {                                                                \
      _Pragma("unroll") for (int c = 0; c < CH; ++c) asm volatile(body : "+v"(acc[c]) : "v"(a), "s"(b)); \
    }                                                                                                \
    uint32_t s = 0;                                                                                  \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) s ^= acc[c];                                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                                  \
  }
K32(k_add, "v_add_u32_e32 %0, %0, %1")
K32(k_add_lit, "v_add_u32_e32 %0, 0x7ffffda, %0")
K32(k_add_sgpr, "v_add_u32_e32 %0, %2, %0")
K32(k_add_self, "v_add_u32_e32 %0, %0, %0")
K32(k_and_lit, "v_and_b32_e32 %0, 0x3ffffff, %0")
K32(k_or, "v_or_b32_e32 %0, %0, %1")
K32(k_lshrrev, "v_lshrrev_b32_e32 %0, 26, %0")
K32(k_lshlrev, "v_lshlrev_b32_e32 %0, 1, %0")
K32(k_not, "v_not_b32_e32 %0, %0")
K32(k_mul_u24, "v_mul_u32_u24_e32 %0, 19, %0")
K32(k_mul_lo19, "v_mul_lo_u32 %0, %0, 19")
K32(k_max, "v_max_u32_e32 %0, %0, %1")
K32(k_subrev, "v_subrev_u32_e32 %0, %0, %1")
K32(k_add3, "v_add3_u32 %0, %0, %1, %1")
K32(k_lshl_add, "v_lshl_add_u32 %0, %0, 1, %1")
K32(k_bitop3, "v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96")
K32(k_and_or, "v_and_or_b32 %0, %0, %1, %1")
K32(k_add_e64, "v_add_u32_e64 %0, %0, %1")
K32(k_xad, "v_xad_u32 %0, %0, %1, %1")
K32(k_pk_add_u16, "v_pk_add_u16 %0, %0, %1")
typedef void (*kfn)(uint64_t*, uint32_t);
int main() {
  const int blocks = 256 * 8, threads = 256;
  uint64_t* d; (void)hipMalloc(&d, sizeof(uint64_t) * blocks * threads);
  struct { const char* name; kfn f; } ks[] = {
    {"v_add_u32_e32", k_add}, {"v_add_u32_e32 literal", k_add_lit}, {"v_add_u32_e32 sgpr", k_add_sgpr},
    {"v_add_u32_e32 x+x", k_add_self}, {"v_and_b32_e32 literal", k_and_lit}, {"v_or_b32_e32", k_or},
    {"v_lshrrev_b32_e32", k_lshrrev}, {"v_lshlrev_b32_e32", k_lshlrev}, {"v_not_b32", k_not},
    {"v_mul_u32_u24_e32 19", k_mul_u24}, {"v_mul_lo_u32 19", k_mul_lo19}, {"v_max_u32_e32", k_max},
    {"v_subrev_u32_e32", k_subrev}, {"v_add3_u32", k_add3}, {"v_lshl_add_u32", k_lshl_add},
    {"v_bitop3_b32", k_bitop3}, {"v_and_or_b32", k_and_or}, {"v_add_u32_e64", k_add_e64}, {"v_xad_u32", k_xad},
    {"v_pk_add_u16", k_pk_add_u16}};
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, (uint32_t)r);
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
    }
    double winst = (double)blocks * threads / 64 * ITERS * CH;  // wave-instructions
    printf("%-24s %7.3f ms  %6.2f T lane-ops/s  %5.2f cycles/wave-instr/SIMD @2.3GHz\n", k.name, best,
           winst * 64 / (best * 1e-3) / 1e12, (best * 1e-3 * 2.3e9 * 1024) / winst);
  }
  return 0;
}
