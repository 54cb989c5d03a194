// v_mad_u64_u32 dependent-chain latency vs independent chains, at 1 and 2 waves/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 8192
template <int CH>
__global__ void k(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed, b = a ^ 0x9e3779b9u;
  uint64_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = (uint64_t)a * b + acc[c];
    a += 1;
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int CH>
void run(uint64_t* d, int wps) {
  const int threads = 256, blocks = 256 * wps;  // wps waves per SIMD
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k<CH>, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k<CH>, dim3(blocks), dim3(threads), 0, 0, d, 2u);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  double mads = (double)blocks * threads * ITERS * CH;
  double per_simd_cycles = ms * 1e-3 * 2.3e9;
  double mads_per_wave_per_cycle = mads / 64.0 / 1024.0 / per_simd_cycles;
  printf("chains=%2d waves/SIMD=%d  %.3f ms  %.2f T mad/s  cycles per wave-mad per SIMD = %.2f\n", CH, wps, ms,
         mads / (ms * 1e-3) / 1e12, 1.0 / mads_per_wave_per_cycle);
}
int main() {
  uint64_t* d; (void)hipMalloc(&d, sizeof(uint64_t) * 256 * 8 * 256);
  for (int w = 1; w <= 4; w *= 2) { run<1>(d, w); run<2>(d, w); run<4>(d, w); run<8>(d, w); }
  return 0;
}
