// Dependent-chain latencies on gfx950, one wave per SIMD (the finish's inversion regime): cycles per link of a
// chain of (a) ds_read_b64 whose address is the previous result, (b) v_add_u32, (c) v_mad_u64_u32,
// (d) v_mul_i32_i24, (e) v_bfe_i32, (f) ds_read_b64 + 5 dependent v_add_u32 (one divstep lookup's shape),
// (g) v_mov_b32_dpp row_newbcast.  s_memtime around 256 links, median over the waves.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench/dep_latency tools/microbench/dep_latency.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define LINKS 256

template <int KIND>
__global__ __launch_bounds__(256) void chain(const uint32_t* seed, uint64_t* out) {
  __shared__ uint64_t tab[2048];
  for (int i = threadIdx.x; i < 2048; i += 256) tab[i] = (uint64_t)((i * 8 + 8) & 0x3FF8);  // next byte offset
  __syncthreads();
  uint32_t x = seed[threadIdx.x & 63] & 0x3FF8;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  asm volatile("" : "+v"(x));
#pragma unroll 1
  for (int i = 0; i < LINKS / 8; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if constexpr (KIND == 0) {
        x = (uint32_t)*(const uint64_t*)((const char*)tab + x);
      } else if constexpr (KIND == 1) {
        asm volatile("v_add_u32 %0, %0, 7" : "+v"(x));
      } else if constexpr (KIND == 2) {
        uint64_t d;
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, 0" : "=v"(d) : "v"(x) : "vcc");
        x = (uint32_t)d;
      } else if constexpr (KIND == 3) {
        asm volatile("v_mul_i32_i24 %0, %0, 3" : "+v"(x));
      } else if constexpr (KIND == 4) {
        asm volatile("v_bfe_i32 %0, %0, 1, 24" : "+v"(x));
      } else if constexpr (KIND == 5) {
        x = (uint32_t)*(const uint64_t*)((const char*)tab + x);
        asm volatile("v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, -1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, -1\n"
                     " v_and_b32_e32 %0, 0x3ff8, %0" : "+v"(x));
      } else {
        x = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x150, 0xF, 0xF, false);
      }
    }
  }
  asm volatile("" : "+v"(x));
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
  if (x == 0xFFFFFFFFu) out[0] = x;  // keep the chain live
}

template <int KIND>
static double run(const uint32_t* dseed, uint64_t* dout, int blocks) {
  hipLaunchKernelGGL(chain<KIND>, dim3(blocks), dim3(256), 0, 0, dseed, dout);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(chain<KIND>, dim3(blocks), dim3(256), 0, 0, dseed, dout);
  hipDeviceSynchronize();
  std::vector<uint64_t> h(blocks * 4);
  hipMemcpy(h.data(), dout, h.size() * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  return (double)h[h.size() / 2] / LINKS;
}

int main() {
  uint32_t* dseed;
  uint64_t* dout;
  const int blocks = 256;  // one block of 4 waves per CU: one wave per SIMD
  hipMalloc(&dseed, 64 * 4);
  hipMalloc(&dout, blocks * 4 * 8);
  std::vector<uint32_t> s(64);
  for (int i = 0; i < 64; ++i) s[i] = (uint32_t)(i / 16) * 64;
  hipMemcpy(dseed, s.data(), 256, hipMemcpyHostToDevice);
  printf("cycles per dependent link (s_memtime = shader cycles), one wave per SIMD:\n");
  printf("  ds_read_b64 (address = previous result)  %.1f\n", run<0>(dseed, dout, blocks));
  printf("  v_add_u32                                %.1f\n", run<1>(dseed, dout, blocks));
  printf("  v_mad_u64_u32                            %.1f\n", run<2>(dseed, dout, blocks));
  printf("  v_mul_i32_i24                            %.1f\n", run<3>(dseed, dout, blocks));
  printf("  v_bfe_i32                                %.1f\n", run<4>(dseed, dout, blocks));
  printf("  ds_read_b64 + 5 dependent VALU           %.1f\n", run<5>(dseed, dout, blocks));
  printf("  v_mov_b32_dpp row_newbcast               %.1f\n", run<6>(dseed, dout, blocks));
  return 0;
}
