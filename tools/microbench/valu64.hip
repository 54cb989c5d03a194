// Issue cost of the 64-bit VALU ops the comb step's carry chains use (v_lshrrev_b64: 63 per step) against the
// 32-bit alternatives (v_alignbit_b32 + v_lshrrev_b32), and of a whole carry extraction both ways in a mad chain.
// Same harness as valu_mix2.hip: 8 independent chains per lane, 2048 blocks x 256 threads, best of 3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 16384
#define CH 8
#define K64(name, body)                                                                              \
  __global__ void name(uint64_t* out, uint32_t seed) {                                               \
    uint64_t acc[CH];                                                                                \
    const uint32_t a = threadIdx.x * 2654435761u + seed;                                             \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) acc[c] = ((uint64_t)a << 20) + c;                 \
    for (int i = 0; i < ITERS; ++i) {                                                                \
      _Pragma("unroll") for (int c = 0; c < CH; ++c) asm volatile(body : "+v"(acc[c]) : "v"(a));     \
    }                                                                                                \
    uint64_t s = 0;                                                                                  \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) s ^= acc[c];                                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                                  \
  }
K64(k_lshr64, "v_lshrrev_b64 %0, 26, %0")
K64(k_lshl_add64, "v_lshl_add_u64 %0, %0, 0, %0")
K64(k_mad, "v_mad_u64_u32 %0, vcc, %1, %1, %0")
// carry extraction of a 64-bit column: limb = lo & M26, carry = acc >> 26 (64-bit), then the next column's mad
#define KC(name, CARRY)                                                                              \
  __global__ void name(uint64_t* out, uint32_t seed) {                                               \
    uint64_t acc[CH];                                                                                \
    uint32_t lsum = 0;                                                                               \
    const uint32_t a = threadIdx.x * 2654435761u + seed;                                             \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) acc[c] = ((uint64_t)a << 20) + c;                 \
    for (int i = 0; i < ITERS; ++i) {                                                                \
      _Pragma("unroll") for (int c = 0; c < CH; ++c) {                                               \
        uint32_t l;                                                                                  \
        asm volatile("v_and_b32_e32 %0, 0x3ffffff, %1" : "=v"(l) : "v"((uint32_t)acc[c]));          \
        lsum += l;                                                                                   \
        CARRY;                                                                                       \
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(acc[c]) : "v"(a));                  \
      }                                                                                              \
    }                                                                                                \
    uint64_t s = lsum;                                                                               \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) s ^= acc[c];                                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                                  \
  }
__device__ __forceinline__ void carry64(uint64_t& x) { asm volatile("v_lshrrev_b64 %0, 26, %0" : "+v"(x)); }
__device__ __forceinline__ void carry32(uint64_t& x) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32), nl, nh;
  asm volatile("v_alignbit_b32 %0, %1, %2, 26" : "=v"(nl) : "v"(hi), "v"(lo));
  asm volatile("v_lshrrev_b32_e32 %0, 26, %1" : "=v"(nh) : "v"(hi));
  x = ((uint64_t)nh << 32) | nl;
}
KC(k_carry64, carry64(acc[c]))
KC(k_carry32, carry32(acc[c]))
typedef void (*kfn)(uint64_t*, uint32_t);
int main() {
  const int blocks = 256 * 8, threads = 256;
  uint64_t* d; (void)hipMalloc(&d, sizeof(uint64_t) * blocks * threads);
  struct { const char* name; kfn f; int ops; } ks[] = {
    {"v_lshrrev_b64", k_lshr64, 1}, {"v_lshl_add_u64", k_lshl_add64, 1}, {"v_mad_u64_u32", k_mad, 1},
    {"and + lshrrev_b64 + mad (+ add)", k_carry64, 3}, {"and + alignbit + lshrrev_b32 + mad (+ add)", k_carry32, 4}};
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, (uint32_t)r);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    // wave-instruction groups per SIMD: blocks * 4 waves * ITERS * CH over 1024 SIMDs
    const double groups = (double)blocks * 4 * ITERS * CH / 1024.0;
    printf("%-42s %8.3f ms  %6.2f ns per group per SIMD (%d ops)\n", k.name, best, best * 1e6 / groups, k.ops);
  }
  return 0;
}
