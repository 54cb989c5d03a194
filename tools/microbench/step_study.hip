// ONE comb step in isolation, at 4 waves per SIMD (1024 blocks x 256 threads, launch bounds
// 256 x 4 = the comb's 128-VGPR budget), against the alternatives the verdict named:
//   step_T      the product's mixed addition (verify_core.h ge_madd_ab<WITH_T = true, CHAIN = true>: 7 products)
//   step_noT    the same without T3 (6 products): what skipping T saves per step -- the comb's LAST step already
//               skips it (verify_kernels.h), and its first step converts the entry with ge_from_ab, whose T the
//               second step reads, so (a) has nothing left to take
//   mul7_r25    the step's 7 products alone, radix 2^25.5 single-chain form (fe_mul_chain<3> + <4>)
//   mul7_r32    the same 7 products in saturated radix 2^32, 8 limbs, product scanning: per product 64
//               v_mad_u64_u32 with carry-out + 64 v_addc_co_u32 into a 96-bit column accumulator, then the
//               fold by 38 (2^256 = 38 mod p) and two short carry passes (verdict item (b))
//   check       mul_r32 vs fe_mul on 2^16 random operand pairs (canonical words equal): the r32 form is exact
// Reported: ns per iteration per SIMD (4 waves sharing it) and shader cycles per iteration per wave at the
// clock measured in-kernel (s_memtime / s_memrealtime), best of 5.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../pbft_amd/csrc/verify_kernels.h"

using namespace pbft;

#define ITERS 2048
#define WAVES_PER_EU 4

struct f32 { uint32_t w[8]; };

// acc (64-bit) + hi (32-bit) += a * b: one mad with carry-out, one add of the carry into the third word
__device__ __forceinline__ void mac2(uint64_t& acc, uint32_t& hi, uint32_t a, uint32_t b) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
      "v_addc_co_u32_e64 %2, %1, %2, 0, %1"
      : "+v"(acc), "=&s"(cc), "+v"(hi) : "v"(a), "v"(b));
}

// N independent products h[m] = f[m] g[m] mod p, values < 2^256 (weakly reduced), interleaved term by term
template <int N>
__device__ __forceinline__ void fe32_mul_n(f32* const h[], const f32* const f[], const f32* const g[]) {
  uint64_t acc[N];
  uint32_t hi[N], w[N][16];
#pragma unroll
  for (int m = 0; m < N; ++m) { acc[m] = 0; hi[m] = 0; }
#pragma unroll
  for (int k = 0; k < 15; ++k) {
#pragma unroll
    for (int i = (k > 7 ? k - 7 : 0); i <= (k < 7 ? k : 7); ++i) {
#pragma unroll
      for (int m = 0; m < N; ++m) mac2(acc[m], hi[m], f[m]->w[i], g[m]->w[k - i]);
    }
#pragma unroll
    for (int m = 0; m < N; ++m) {
      w[m][k] = (uint32_t)acc[m];
      acc[m] = (acc[m] >> 32) | ((uint64_t)hi[m] << 32);
      hi[m] = 0;
    }
  }
#pragma unroll
  for (int m = 0; m < N; ++m) {
    w[m][15] = (uint32_t)acc[m];
    uint32_t o[8];
    uint64_t t = 0;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      t = (uint64_t)38u * w[m][8 + i] + ((uint64_t)w[m][i] + c);
      o[i] = (uint32_t)t;
      c = (uint32_t)(t >> 32);
    }
    t = (uint64_t)38u * c + o[0];  // c < 39
    o[0] = (uint32_t)t;
    uint32_t cy = (uint32_t)(t >> 32);
#pragma unroll
    for (int i = 1; i < 8; ++i) {
      const uint64_t u = (uint64_t)o[i] + cy;
      o[i] = (uint32_t)u;
      cy = (uint32_t)(u >> 32);
    }
    o[0] += 38u * cy;  // (wrapped past 2^256: o[0] < 2^12 here, no further carry)
#pragma unroll
    for (int i = 0; i < 8; ++i) h[m]->w[i] = o[i];
  }
}

__device__ __forceinline__ void perturb(fe& a, uint32_t it) { a.v[0] ^= it & 7u; }
__device__ __forceinline__ void perturb32(f32& a, uint32_t it) { a.w[0] ^= it & 7u; }

// The comb's loop body exactly (verify_kernels.h comb_kernel, chain form): the lane's gathered entry read from its
// LDS buffer with the sign picked by address (lds_entry_signed), lgkmcnt(0), the mixed addition, the limbs laundered.
template <bool WITH_T>
__global__ void __launch_bounds__(256, WAVES_PER_EU) k_step(uint32_t* out, uint64_t* clk, uint32_t seed) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t ebuf = (uint32_t)(uintptr_t)lds + wave * COMB_LDS_PER_WAVE;
  const uint32_t rd0 = ebuf + 128u * lane + 16u * (lane & 7);
  const uint32_t x = threadIdx.x * 2654435761u + blockIdx.x * 40503u + seed;
  for (uint32_t o = 0; o < 128; o += 4) lds_write32(rd0 ^ o, (x * (o + 11u) >> (o % 7)) & M25);
  __syncthreads();
  ge P;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    P.X.v[i] = (x >> i) & M25; P.Y.v[i] = (x * 3u >> i) & M25; P.Z.v[i] = (x * 5u >> i) & M25;
    P.T.v[i] = (x * 7u >> i) & M25;
  }
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < ITERS; ++it) {
    fe qa, qb, k;
    const bool neg = (it & 1) != 0;
    lds_entry_signed(rd0, neg, qa, qb, k);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    ge_madd_ab<WITH_T, true>(P, P, qa, qb, k, neg);
#pragma unroll
    for (int t = 0; t < 10; ++t) asm("" : "+v"(P.X.v[t]), "+v"(P.Y.v[t]), "+v"(P.Z.v[t]), "+v"(P.T.v[t]));
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) s ^= P.X.v[i] ^ P.Y.v[i] ^ P.Z.v[i] ^ P.T.v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

__global__ void __launch_bounds__(256, 2) k_mul7_r25(uint32_t* out, uint64_t* clk, uint32_t seed) {
  const uint32_t x = threadIdx.x * 2654435761u + blockIdx.x * 40503u + seed;
  fe a, b, c, d, e, f, g, q0, q1, q2;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    a.v[i] = (x >> i) & M25; b.v[i] = (x * 3u >> i) & M25; c.v[i] = (x * 5u >> i) & M25;
    q0.v[i] = (x * 7u >> i) & M25; q1.v[i] = (x * 11u >> i) & M25; q2.v[i] = (x * 13u >> i) & M25;
  }
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < ITERS; ++it) {
    perturb(q0, it);
    {
      fe* const ho[3] = {&d, &e, &f};
      const fe* const fo[3] = {&a, &b, &c};
      const fe* const go[3] = {&q0, &q1, &q2};
      fe_mul_chain<3>(ho, fo, go);
    }
    {
      fe* const ho[4] = {&a, &b, &c, &g};
      const fe* const fo[4] = {&d, &e, &d, &f};
      const fe* const go[4] = {&f, &d, &e, &e};
      fe_mul_chain<4>(ho, fo, go);
    }
    b.v[0] ^= g.v[1];
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) s ^= a.v[i] ^ b.v[i] ^ c.v[i] ^ g.v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

__global__ void __launch_bounds__(256, 2) k_mul7_r32(uint32_t* out, uint64_t* clk, uint32_t seed) {
  const uint32_t x = threadIdx.x * 2654435761u + blockIdx.x * 40503u + seed;
  f32 a, b, c, d, e, f, g, q0, q1, q2;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a.w[i] = x * (2u * i + 1u); b.w[i] = x * 3u + i; c.w[i] = x ^ (5u * i);
    q0.w[i] = x * 7u + 3u * i; q1.w[i] = x * 11u - i; q2.w[i] = x * 13u ^ i;
  }
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < ITERS; ++it) {
    perturb32(q0, it);
    {
      f32* const ho[3] = {&d, &e, &f};
      const f32* const fo[3] = {&a, &b, &c};
      const f32* const go[3] = {&q0, &q1, &q2};
      fe32_mul_n<3>(ho, fo, go);
    }
    {
      f32* const ho[4] = {&a, &b, &c, &g};
      const f32* const fo[4] = {&d, &e, &d, &f};
      const f32* const go[4] = {&f, &d, &e, &e};
      fe32_mul_n<4>(ho, fo, go);
    }
    b.w[0] ^= g.w[1];
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= a.w[i] ^ b.w[i] ^ c.w[i] ^ g.w[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

// correctness: r32 product vs fe_mul, as canonical words
__global__ void k_check(const uint32_t* A, const uint32_t* B, uint32_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  f32 a, b, h;
  for (int t = 0; t < 8; ++t) { a.w[t] = A[8 * i + t]; b.w[t] = B[8 * i + t]; }
  f32* ho[1] = {&h};
  const f32* fo[1] = {&a};
  const f32* go[1] = {&b};
  fe32_mul_n<1>(ho, fo, go);
  // h (< 2^256) -> canonical via the radix-2^25.5 path: h = hl + 2^255 hb  ==  hl + 19 hb
  uint32_t wl[8];
  for (int t = 0; t < 8; ++t) wl[t] = h.w[t];
  const uint32_t top = wl[7] >> 31;
  wl[7] &= 0x7fffffffu;
  fe x, y, r, nineteen;
  fe_from_words(x, wl);
  fe_zero(nineteen); nineteen.v[0] = 19u * top;
  fe_add(x, x, nineteen);
  uint32_t aw[8], bw[8];
  for (int t = 0; t < 8; ++t) { aw[t] = a.w[t]; bw[t] = b.w[t]; }
  const uint32_t at = aw[7] >> 31, bt = bw[7] >> 31;
  aw[7] &= 0x7fffffffu; bw[7] &= 0x7fffffffu;
  fe fa, fb, t19;
  fe_from_words(fa, aw); fe_from_words(fb, bw);
  fe_zero(t19); t19.v[0] = 19u * at; fe_add(fa, fa, t19); fe_carry(fa);
  fe_zero(t19); t19.v[0] = 19u * bt; fe_add(fb, fb, t19); fe_carry(fb);
  fe_mul(y, fa, fb);
  fe_carry(x);
  uint32_t wx[8], wy[8];
  fe_to_words(wx, x);
  fe_to_words(wy, y);
  uint32_t ok = 1;
  for (int t = 0; t < 8; ++t) ok &= wx[t] == wy[t];
  (void)r;
  out[i] = ok;
}

typedef void (*kfn)(uint32_t*, uint64_t*, uint32_t);
// (the 7-product kernels hold 10 field elements: compiled and launched at 2 waves per SIMD, 256 VGPRs, no spill,
// both radices alike)
int main() {
  const int blocks = 1024, threads = 256;  // 4 blocks per CU on 256 CUs: 4 waves per SIMD
  uint32_t* d;
  uint64_t* dc;
  (void)hipMalloc(&d, sizeof(uint32_t) * blocks * threads);
  (void)hipMalloc(&dc, 16);
  // correctness of the r32 form
  {
    const int n = 1 << 16;
    std::mt19937_64 rng(5);
    std::vector<uint32_t> A(8 * n), B(8 * n), ok(n);
    for (auto& v : A) v = (uint32_t)rng();
    for (auto& v : B) v = (uint32_t)rng();
    for (int i = 0; i < 64; ++i) for (int t = 0; t < 8; ++t) { A[8 * i + t] = 0xffffffffu; B[8 * i + t] = i & 1 ? 0xffffffffu : (uint32_t)rng(); }
    uint32_t *dA, *dB, *dO;
    (void)hipMalloc(&dA, 32 * n); (void)hipMalloc(&dB, 32 * n); (void)hipMalloc(&dO, 4 * n);
    (void)hipMemcpy(dA, A.data(), 32 * n, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, B.data(), 32 * n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, dA, dB, dO, n);
    (void)hipMemcpy(ok.data(), dO, 4 * n, hipMemcpyDeviceToHost);
    int good = 0;
    for (int i = 0; i < n; ++i) good += ok[i];
    printf("check: radix-2^32 product == fe_mul on %d / %d operand pairs (64 with all-ones words)\n", good, n);
  }
  struct { const char* name; kfn f; int waves; unsigned lds; } ks[] = {
      {"step_T   (ge_madd_ab, 7 products, the comb's step)", k_step<true>, WAVES_PER_EU, 4 * COMB_LDS_PER_WAVE},
      {"step_noT (6 products, no T3)", k_step<false>, WAVES_PER_EU, 4 * COMB_LDS_PER_WAVE},
      {"mul7_r25 (7 products, radix 2^25.5 chains)", k_mul7_r25, 2, 0},
      {"mul7_r32 (7 products, radix 2^32, 8 limbs)", k_mul7_r32, 2, 0}};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (auto& k : ks) {
    const int kb = blocks * k.waves / WAVES_PER_EU;
    hipLaunchKernelGGL(k.f, dim3(kb), dim3(threads), k.lds, 0, d, dc, 1u);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    uint64_t clk[2] = {0, 0}, bclk[2] = {0, 0};
    for (int r = 0; r < 5; ++r) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(kb), dim3(threads), k.lds, 0, d, dc, (uint32_t)r + 2);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      (void)hipMemcpy(clk, dc, 16, hipMemcpyDeviceToHost);
      if (ms < best) { best = ms; bclk[0] = clk[0]; bclk[1] = clk[1]; }
    }
    // every SIMD runs k.waves waves x ITERS iterations; cycles per iteration per wave from wave 0's own clock
    const double ns_simd = best * 1e6 / ((double)k.waves * ITERS);
    const double ghz = bclk[1] ? (double)bclk[0] / (bclk[1] * 10.0) : 0.0;  // s_memrealtime: 100 MHz
    printf("%-52s %d waves/SIMD %8.3f ms  %7.1f ns/iter/SIMD  %7.0f cycles/iter/wave at %.2f GHz\n", k.name,
           k.waves, best, ns_simd, (double)bclk[0] / ITERS, ghz);
  }
  return 0;
}
