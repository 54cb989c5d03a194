// v_mad_u64_u32 latency and throughput with the interleaving pinned by inline asm (the compiler otherwise
// serialises or fuses chains: tools/microbench/mad_latency.hip measured a*b hoisted out of its chains).
// CH independent accumulators, one mad of each in turn, 16 rounds per asm block; every wave stamps
// s_memtime around its loop, so the result is shader cycles per wave-mad, whatever the clock.
// Grid: 1024 x W single-wave blocks = W waves per SIMD on 256 CUs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define ITERS 2048
#define M1(c) "v_mad_u64_u32 %" #c ", vcc, %[x], %[y], %" #c "\n\t"

template <int CH>
__global__ void k(uint64_t* out, uint64_t* cyc, uint32_t seed) {
  uint32_t x = threadIdx.x * 2654435761u + seed, y = x ^ 0x9e3779b9u;
  uint64_t a0 = x, a1 = x + 1, a2 = x + 2, a3 = x + 3, a4 = x + 4, a5 = x + 5, a6 = x + 6, a7 = x + 7;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; ++i) {
    if constexpr (CH == 1) {
      asm volatile(M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0)
                   : "+v"(a0) : [x] "v"(x), [y] "v"(y) : "vcc");
    } else if constexpr (CH == 2) {
#define R2 M1(0) M1(1)
      asm volatile(R2 R2 R2 R2 R2 R2 R2 R2 R2 R2 R2 R2 R2 R2 R2 R2 : "+v"(a0), "+v"(a1) : [x] "v"(x), [y] "v"(y) : "vcc");
    } else if constexpr (CH == 3) {
#define R3 M1(0) M1(1) M1(2)
      asm volatile(R3 R3 R3 R3 R3 R3 R3 R3 R3 R3 R3 R3 R3 R3 R3 R3
                   : "+v"(a0), "+v"(a1), "+v"(a2) : [x] "v"(x), [y] "v"(y) : "vcc");
    } else if constexpr (CH == 4) {
#define R4 M1(0) M1(1) M1(2) M1(3)
      asm volatile(R4 R4 R4 R4 R4 R4 R4 R4 R4 R4 R4 R4 R4 R4 R4 R4
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : [x] "v"(x), [y] "v"(y) : "vcc");
    } else if constexpr (CH == 101) {  // one chain, s_nop 0 after every mad (the asm-boundary pad)
#define MN M1(0) "s_nop 0\n\t"
      asm volatile(MN MN MN MN MN MN MN MN MN MN MN MN MN MN MN MN : "+v"(a0) : [x] "v"(x), [y] "v"(y) : "vcc");
    } else if constexpr (CH == 102) {  // two chains, s_nop 0 after every second mad
#define MN2 M1(0) M1(1) "s_nop 0\n\t"
      asm volatile(MN2 MN2 MN2 MN2 MN2 MN2 MN2 MN2 : "+v"(a0), "+v"(a1) : [x] "v"(x), [y] "v"(y) : "vcc");
    } else {
#define R8 M1(0) M1(1) M1(2) M1(3) M1(4) M1(5) M1(6) M1(7)
      asm volatile(R8 R8 R8 R8 R8 R8 R8 R8 R8 R8 R8 R8 R8 R8 R8 R8
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : [x] "v"(x), [y] "v"(y) : "vcc");
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CH>
void run(uint64_t* d, uint64_t* dc, int wps) {
  const int blocks = 1024 * wps;
  hipLaunchKernelGGL(k<CH>, dim3(blocks), dim3(64), 0, 0, d, dc, 1u);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k<CH>, dim3(blocks), dim3(64), 0, 0, d, dc, 2u);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<uint64_t> c(blocks);
  (void)hipMemcpy(c.data(), dc, blocks * 8, hipMemcpyDeviceToHost);
  std::sort(c.begin(), c.end());
  const double mads_per_wave = (double)ITERS * 16 * (CH == 101 ? 1 : CH == 102 ? 1 : CH);
  const double med = (double)c[blocks / 2];
  const double wall_mads = (double)blocks * 64 * mads_per_wave;
  printf("chains=%d waves/SIMD=%d  cycles per mad in a wave %.2f  per SIMD %.2f  (%.3f ms, %.2f T mad/s)\n", CH, wps,
         med / mads_per_wave, med / mads_per_wave / wps, ms, wall_mads / (ms * 1e-3) / 1e12);
}

int main() {
  uint64_t *d, *dc;
  (void)hipMalloc(&d, sizeof(uint64_t) * 1024 * 8 * 64);
  (void)hipMalloc(&dc, sizeof(uint64_t) * 1024 * 8);
  for (int w = 1; w <= 4; w *= 2) { run<1>(d, dc, w); run<2>(d, dc, w); run<3>(d, dc, w); run<4>(d, dc, w); run<8>(d, dc, w); run<101>(d, dc, w); run<102>(d, dc, w); }
  return 0;
}
