// Microbenchmark: per-instruction throughput of the integer ops a GF(2^255-19)
// field multiply can be built from, on gfx950. Each kernel runs 8 independent
// dependency chains per lane so issue throughput (not latency) is measured.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 32768
#define CH 8

__global__ void k_mad64(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed, b = a ^ 0x9e3779b9u;
  uint64_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b) : "s0", "s1");
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mullo(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(a));
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mulhi(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(a));
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul24(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(acc[c]) : "v"(a));
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mulhi24(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(acc[c]) : "v"(a));
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_add(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(a));
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_add3(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(acc[c]) : "v"(a));
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_lshl_add(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(acc[c]) : "v"(a));
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma64(uint64_t* out, uint32_t seed) {
  double a = (double)(threadIdx.x + seed) * 1e-9;
  double acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(acc[c]) : "v"(a));
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

__global__ void k_fma32(uint64_t* out, uint32_t seed) {
  float a = (float)(threadIdx.x + seed) * 1e-9f;
  float acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(acc[c]) : "v"(a));
  }
  float s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

__global__ void k_addc(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(acc[c]) : "v"(a) : "vcc");
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(uint64_t*, uint32_t);
int main() {
  const int blocks = 256 * 8, threads = 256;
  uint64_t* d; hipMalloc(&d, sizeof(uint64_t) * blocks * threads);
  struct { const char* name; kfn f; } ks[] = {
    {"v_mad_u64_u32", k_mad64}, {"v_mul_lo_u32", k_mullo}, {"v_mul_hi_u32", k_mulhi},
    {"v_mad_u32_u24", k_mul24}, {"v_mul_hi_u32_u24", k_mulhi24}, {"v_add_u32", k_add},
    {"v_add3_u32", k_add3}, {"v_alignbit_b32", k_lshl_add}, {"v_fma_f64", k_fma64},
    {"v_fma_f32", k_fma32}, {"v_addc_co_u32(vcc chain)", k_addc}};
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, (uint32_t)r);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
    }
    double ops = (double)blocks * threads * ITERS * CH;
    printf("%-28s %8.3f ms  %8.2f Tlane-ops/s  (%.1f lane-ops/clk/CU @2.4GHz)\n", k.name, best,
           ops / (best * 1e-3) / 1e12, ops / (best * 1e-3) / 2.4e9 / 256);
  }
  return 0;
}
