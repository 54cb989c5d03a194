// Batch-inversion finish of the one-lane-per-signature verify (comb_kernel ->
// finish_kernel), its own translation unit.
#include <hip/hip_runtime.h>
#include <stdint.h>

// (before verify_kernels.h: finish_core.h, which it includes, expands FIN_STAMP)
#ifndef PBFT_FIN_STAMPS
#define PBFT_FIN_STAMPS 0  // 1: timing build -- every wave stamps s_memtime at its phase boundaries
#endif
#if PBFT_FIN_STAMPS
#define FIN_STAMP_WAVES 4096
__device__ uint64_t g_fin_stamp[FIN_STAMP_WAVES][12];
#define FIN_STAMP(k) \
  if (lane == 0 && wave < FIN_STAMP_WAVES) g_fin_stamp[wave][k] = __builtin_amdgcn_s_memtime()
extern "C" int pbft_debug_fin_stamps(uint64_t* out, uint32_t waves) {
  if (waves > FIN_STAMP_WAVES) waves = FIN_STAMP_WAVES;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fin_stamp), sizeof(uint64_t) * 12 * waves, 0,
                                  hipMemcpyDeviceToHost);
}
#else
#define FIN_STAMP(k)
#endif
#include "verify_kernels.h"


// W: waves per SIMD the kernel is compiled for (register budget 512 / W); the prefetch of X, Y, Z needs W = 1
template <int FM, int LV, int W>
__global__ void __launch_bounds__(BLOCK, W) finish_kernel(const uint8_t* __restrict__ R,
                                                       uint32_t rs_stride,
                                                       const uint32_t* __restrict__ xyz,
                                                       const uint8_t* __restrict__ flags, uint64_t N,
                                                       uint64_t* __restrict__ bitmap) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;
  // PRE: small FM keeps every Z and issues the X, Y loads before the inversion, so the back-substitution
  // does not wait on memory (FM <= 4: ~100 more VGPRs, within the 2-waves-per-SIMD budget)
  constexpr bool PRE = PBFT_FIN_PREFETCH && ((FM <= 4 && W == 1) || FM == 1);
#if FIN_USE_TAB
  // LV > 0: the divstep table (inv25519.h) goes to LDS; every wave of the block copies its share and meets the
  // one barrier before the inversion (waves past N included, so the barrier count always matches)
  __shared__ uint64_t ds_tab[LV > 0 ? DS_TAB_ENTRIES : 1];
  if constexpr (LV > 0) {
    const uint4* src = (const uint4*)g_ds_tab.e;
    uint4* dst = (uint4*)ds_tab;
#pragma unroll
    for (int k = 0; k < DS_TAB_ENTRIES / 2 / BLOCK; ++k) dst[k * BLOCK + threadIdx.x] = src[k * BLOCK + threadIdx.x];
    if (wave * FM * 64 >= N) { __syncthreads(); return; }
  }
#else
  const uint64_t* ds_tab = nullptr;
#endif
  if (wave * FM * 64 >= N) return;
  finish_wave<FM, LV, PRE, true>(wave, lane, R, rs_stride, xyz, flags, N, bitmap, ds_tab);
}


hipError_t launch_finish(int fm, int lv, int w, const uint8_t* R, uint32_t rs_stride, const uint32_t* xyz,
                         const uint8_t* flags, uint64_t N, uint64_t* bitmap, hipStream_t st) {
#define PBFT_LAUNCH_FIN(M_, LV_, W_)                                                                           \
  hipLaunchKernelGGL((finish_kernel<M_, LV_, W_>),                                                          \
                     dim3((unsigned)((((N + 64 * M_ - 1) / (64 * M_)) * 64 + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, \
                     st, R, rs_stride, xyz, flags, N, bitmap)
  if (lv == 0) {
    if (fm == 16) PBFT_LAUNCH_FIN(16, 0, FIN_WAVES_PER_EU);
    else if (fm == 8) PBFT_LAUNCH_FIN(8, 0, FIN_WAVES_PER_EU);
    else if (fm == 4) PBFT_LAUNCH_FIN(4, 0, FIN_WAVES_PER_EU);
    else if (fm == 2) PBFT_LAUNCH_FIN(2, 0, FIN_WAVES_PER_EU);
    else PBFT_LAUNCH_FIN(1, 0, FIN_WAVES_PER_EU);
  } else if (w >= 2) {  // product tree at two waves per SIMD (prefetch at width 1 only): large rounds, small shards
    if (fm >= 8) PBFT_LAUNCH_FIN(8, PBFT_FIN_LV, 2);
    else if (fm == 4) PBFT_LAUNCH_FIN(4, PBFT_FIN_LV, 2);
    else if (fm == 2) PBFT_LAUNCH_FIN(2, PBFT_FIN_LV, 2);
    else PBFT_LAUNCH_FIN(1, PBFT_FIN_LV, 2);
  } else {
    if (fm == 16) PBFT_LAUNCH_FIN(16, PBFT_FIN_LV, 1);
    else if (fm == 8) PBFT_LAUNCH_FIN(8, PBFT_FIN_LV, 1);
    else if (fm == 4) PBFT_LAUNCH_FIN(4, PBFT_FIN_LV, 1);
    else if (fm == 2) PBFT_LAUNCH_FIN(2, PBFT_FIN_LV, 1);
    else PBFT_LAUNCH_FIN(1, PBFT_FIN_LV, 1);
  }
#undef PBFT_LAUNCH_FIN
  return hipGetLastError();
}


// ---- test hook: the finish's row-wise inversion on arbitrary values ----------------------------------------
// One value per 16-lane row (so every row of a wave inverts its own value, as in finish_kernel), through the same
// fe_invert_wave<true> and LDS divstep table; tests/test_gpu_verify.py checks it against z^(p-2) on the inversion
// extremes.  Not part of the verify path (and not declared in include/: a test hook, like pbft_debug_fin_stamps).
__global__ void __launch_bounds__(64) debug_invert_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                          uint32_t n) {
  __shared__ uint64_t ds_tab[DS_TAB_ENTRIES];
  {
    const uint4* src = (const uint4*)g_ds_tab.e;
    uint4* dst = (uint4*)ds_tab;
    for (int k = threadIdx.x; k < DS_TAB_ENTRIES / 2; k += 64) dst[k] = src[k];
  }
  __syncthreads();
  const uint32_t row = blockIdx.x * 4 + (threadIdx.x >> 4);
  const uint32_t i = row < n ? row : n - 1;  // (rows past n invert a copy of the last value: uniform per row)
  uint32_t w[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) w[t] = in[(size_t)i * 8 + t];
  fe z, inv;
  fe_from_words(z, w);
  fe_invert_wave<true>(inv, z, ds_tab);
  fe_to_words(w, inv);
  if ((threadIdx.x & 15) == 0 && row < n) {
#pragma unroll
    for (int t = 0; t < 8; ++t) out[(size_t)row * 8 + t] = w[t];
  }
}

// in, out: n values as 8 little-endian 32-bit words each (in < 2^255, any residue; out canonical)
extern "C" int pbft_debug_invert(const uint32_t* in, uint32_t* out, uint32_t n) {
  if (!in || !out || n == 0 || n > (1u << 20)) return -1;
  uint32_t *din = nullptr, *dout = nullptr;
  const size_t bytes = (size_t)n * 32;
  hipError_t e = hipMalloc(&din, bytes);
  if (e == hipSuccess) e = hipMalloc(&dout, bytes);
  if (e == hipSuccess) e = hipMemcpy(din, in, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(debug_invert_kernel, dim3((n + 3) / 4), dim3(64), 0, 0, din, dout, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost);
  if (din) (void)hipFree(din);
  if (dout) (void)hipFree(dout);
  return e == hipSuccess ? 0 : -(int)e - 1;
}
