// RFC 8032 signing kernel (the replicas' own Prepare/Commit envelopes), its own translation unit.
#include "verify_kernels.h"

// RFC 8032 signing, one signature per lane (replicas sign their own
// Prepare/Commit envelopes; the reference multicasts them unsigned).
template <int LEN>
__global__ void __launch_bounds__(BLOCK) sign_kernel(const uint32_t* __restrict__ seeds,
                                                     const uint16_t* __restrict__ seed_idx,
                                                     const uint8_t* __restrict__ msg, uint32_t msg_len,
                                                     uint32_t msg_stride, uint64_t N,
                                                     const uint32_t* __restrict__ tabB, uint32_t* __restrict__ R,
                                                     uint32_t* __restrict__ S, uint32_t* __restrict__ pub,
                                                     uint32_t n_seeds) {
  const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= N) return;
  const uint32_t si = seed_idx[i];
  uint32_t seed[8], r[8], s[8], a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) seed[j] = seeds[8 * si + j];
  sign_lane<PLB, LEN>(r, s, a, seed, msg + (size_t)msg_stride * i, (int)msg_len, tabB);
#pragma unroll
  for (int j = 0; j < 8; ++j) { R[8 * i + j] = r[j]; S[8 * i + j] = s[j]; }
  (void)n_seeds;
  if (pub) {
#pragma unroll
    for (int j = 0; j < 8; ++j) pub[8 * si + j] = a[j];  // identical values from every lane of a seed
  }
}


void launch_sign(int len, dim3 grid, dim3 block, size_t lds, hipStream_t st, const uint32_t* seeds,
                 const uint16_t* seed_idx, const uint8_t* msg, uint32_t msg_len, uint32_t msg_stride, uint64_t N,
                 const uint32_t* tabB, uint32_t* R, uint32_t* S, uint32_t* pub, uint32_t n_seeds) {
  if (len == PBFT_ENVELOPE_LEN)
    hipLaunchKernelGGL(sign_kernel<PBFT_ENVELOPE_LEN>, grid, block, lds, st, seeds, seed_idx, msg, msg_len,
                       msg_stride, N, tabB, R, S, pub, n_seeds);
  else if (len == 0)
    hipLaunchKernelGGL(sign_kernel<0>, grid, block, lds, st, seeds, seed_idx, msg, msg_len, msg_stride, N, tabB, R,
                       S, pub, n_seeds);
  else
    hipLaunchKernelGGL(sign_kernel<-1>, grid, block, lds, st, seeds, seed_idx, msg, msg_len, msg_stride, N, tabB, R,
                       S, pub, n_seeds);
}
