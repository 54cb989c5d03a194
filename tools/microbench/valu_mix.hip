// Throughput of the instructions that dominate verify's ISA (beyond v_mad_u64_u32):
// 64-bit adds/shifts/moves, VOP2 logic, selects, byte permutes.  8 independent chains.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 16384
#define CH 8
#define K32(name, body) K32C(name, body, "vcc")
#define K32N(name, body) K32C(name, body)
#define K32C(name, body, ...)                                                              \
  __global__ void name(uint64_t* out, uint32_t seed) {                               \
    uint32_t a = threadIdx.x * 2654435761u + seed;                                   \
    uint32_t acc[CH];                                                                \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) acc[c] = a + c;                   \
    for (int i = 0; i < ITERS; ++i) {                                                \
      _Pragma("unroll") for (int c = 0; c < CH; ++c) asm volatile(body : "+v"(acc[c]) : "v"(a) : __VA_ARGS__); \
    }                                                                                \
    uint32_t s = 0;                                                                  \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) s ^= acc[c];                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                  \
  }
#define K64(name, body, AT)                                                          \
  __global__ void name(uint64_t* out, uint32_t seed) {                               \
    AT a = threadIdx.x * 2654435761u + seed;                                         \
    uint64_t acc[CH];                                                                \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) acc[c] = a + c;                   \
    for (int i = 0; i < ITERS; ++i) {                                                \
      _Pragma("unroll") for (int c = 0; c < CH; ++c) asm volatile(body : "+v"(acc[c]) : "v"(a) : "vcc"); \
    }                                                                                \
    uint64_t s = 0;                                                                  \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) s ^= acc[c];                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                  \
  }
K64(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 0, %1", uint64_t)
K64(k_lshrrev_b64, "v_lshrrev_b64 %0, 26, %0", uint32_t)
K64(k_mov_b64, "v_mov_b64 %0, %1", uint64_t)
K64(k_mad64, "v_mad_u64_u32 %0, vcc, %1, %1, %0", uint32_t)
K32(k_and_e32, "v_and_b32_e32 %0, %0, %1")
K32(k_xor_e32, "v_xor_b32_e32 %0, %0, %1")
K32(k_add_e32, "v_add_u32_e32 %0, %0, %1")
K32(k_mov_b32, "v_mov_b32_e32 %0, %1")
K32(k_cndmask_e32, "v_cndmask_b32_e32 %0, %0, %1, vcc")
// cndmask without a vcc clobber (the clobber makes the compiler insert hazard nops);
// vcc is set once by a compare outside the loop, as in the verify kernels
K32N(k_cndmask_novcc, "v_cndmask_b32_e32 %0, %0, %1, vcc")
K32(k_perm, "v_perm_b32 %0, %0, %1, %1")
K32(k_bfi, "v_bfi_b32 %0, %0, %1, %1")
K32(k_alignbit, "v_alignbit_b32 %0, %0, %1, 7")
K32(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
K32(k_add_co, "v_add_co_u32_e32 %0, vcc, %0, %1")
K32(k_sub_e32, "v_sub_u32_e32 %0, %0, %1")
K32(k_lshlrev_e32, "v_lshlrev_b32_e32 %0, 1, %0")
// selects: e64 cndmask with an SGPR-pair mask from a compare, and v_bfi with a VGPR lane mask
__global__ void k_cndmask_e64(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed;
  uint32_t acc[CH];
  _Pragma("unroll") for (int c = 0; c < CH; ++c) acc[c] = a + c;
  const uint64_t m = __ballot(a & 1);
  for (int i = 0; i < ITERS; ++i) {
    _Pragma("unroll") for (int c = 0; c < CH; ++c) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(acc[c]) : "v"(a), "s"(m));
  }
  uint32_t s = 0;
  _Pragma("unroll") for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_bfi_sel(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed;
  uint32_t acc[CH];
  _Pragma("unroll") for (int c = 0; c < CH; ++c) acc[c] = a + c;
  const uint32_t m = 0u - (a & 1u);
  for (int i = 0; i < ITERS; ++i) {
    _Pragma("unroll") for (int c = 0; c < CH; ++c) asm volatile("v_bfi_b32 %0, %2, %1, %0" : "+v"(acc[c]) : "v"(a), "v"(m));
  }
  uint32_t s = 0;
  _Pragma("unroll") for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// compiler-generated select from a per-lane predicate (what ge_madd_signed compiles to)
__global__ void k_select_c(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed;
  uint32_t acc[CH];
  _Pragma("unroll") for (int c = 0; c < CH; ++c) acc[c] = a + c;
  const bool neg = a & 1;
  for (int i = 0; i < ITERS; ++i) {
    _Pragma("unroll") for (int c = 0; c < CH; ++c) {
      uint32_t x = neg ? a : acc[c];
      asm volatile("" : "+v"(x));
      acc[c] = x;
    }
  }
  uint32_t s = 0;
  _Pragma("unroll") for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
typedef void (*kfn)(uint64_t*, uint32_t);
int main() {
  const int blocks = 256 * 8, threads = 256;
  uint64_t* d; (void)hipMalloc(&d, sizeof(uint64_t) * blocks * threads);
  struct { const char* name; kfn f; } ks[] = {
    {"v_lshl_add_u64", k_lshl_add_u64}, {"v_lshrrev_b64", k_lshrrev_b64}, {"v_mov_b64", k_mov_b64},
    {"v_mad_u64_u32", k_mad64}, {"v_and_b32_e32", k_and_e32}, {"v_xor_b32_e32", k_xor_e32},
    {"v_add_u32_e32", k_add_e32}, {"v_mov_b32_e32", k_mov_b32}, {"v_cndmask_b32_e32", k_cndmask_e32}, {"v_cndmask_b32_e32 (no clobber)", k_cndmask_novcc},
    {"v_cndmask_b32_e64 sgpr mask", k_cndmask_e64}, {"v_bfi_b32 vgpr lane mask", k_bfi_sel}, {"select (compiler)", k_select_c},
    {"v_perm_b32", k_perm}, {"v_bfi_b32", k_bfi}, {"v_alignbit_b32", k_alignbit}, {"v_mul_lo_u32", k_mul_lo},
    {"v_add_co_u32_e32", k_add_co}, {"v_sub_u32_e32", k_sub_e32}, {"v_lshlrev_b32_e32", k_lshlrev_e32}};
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
    printf("%-22s %7.3f ms  %6.2f T lane-ops/s  %5.2f cycles/wave-instr/SIMD @2.3GHz\n", k.name, best,
           winst * 64 / (best * 1e-3) / 1e12, (best * 1e-3 * 2.3e9 * 1024) / winst);
  }
  return 0;
}
