// Comb-table build kernels (base point and replica keys), one translation unit
// so that they compile in parallel with the verify kernels.
#include "verify_kernels.h"

#define PBFT_HIP_RET(expr)             \
  do {                                 \
    hipError_t _e = (expr);            \
    if (_e != hipSuccess) return _e;   \
  } while (0)

// Comb tables for a set of points given by encoding (negate: tables of -P).
// Pass 1, one thread per (key, position): decompress, key_ok, and the
// position's base point 2^bitoff(pos) * (+-P) by bitoff(pos) doublings.
// slot (optional): key k of this build goes to slot slot[k] of the tables / key_ok / keys_out (a partial
// rebuild, pbft_verify_update_keys); keys_out (optional) receives the raw encodings at their slots.
template <class PL>
__global__ void __launch_bounds__(BLOCK) comb_base_kernel(const uint32_t* __restrict__ enc, uint32_t n_keys,
                                                          int negate, ge* __restrict__ bases,
                                                          uint8_t* __restrict__ dec_ok, uint8_t* __restrict__ key_ok,
                                                          const uint32_t* __restrict__ slot,
                                                          uint32_t* __restrict__ keys_out) {
  constexpr int P = PL::P;
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (uint64_t)P * n_keys) return;
  const uint32_t key = (uint32_t)(tid / P);
  const int pos = (int)(tid % P);
  const uint32_t sl = slot ? slot[key] : key;
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = enc[8 * key + i];
  ge A;
  const bool dec = ge_decompress(A, w);
  if (pos == 0) {
    dec_ok[key] = dec ? 1 : 0;
    if (key_ok) key_ok[sl] = (dec && !ge_is_small_order(A)) ? 1 : 0;
    if (keys_out) {
#pragma unroll
      for (int i = 0; i < 8; ++i) keys_out[8 * sl + i] = w[i];
    }
  }
  if (!dec) ge_identity(A);
  if (negate) { ge t; ge_neg(t, A); A = t; }
  for (int i = 0; i < PL::bitoff(pos); ++i) ge_dbl(A, A);
  bases[tid] = A;
}

// Pass 2, one thread per (key, position, run of TAB_RUN consecutive entries):
// j0 * base by double-and-add, then each next entry by one addition of base;
// the run's TAB_RUN Z coordinates are inverted together (Montgomery's trick:
// 1 inversion + 3 muls each), so an entry costs ~15 field multiplications
// instead of one inversion (~265).  Entry 0 of every position is the identity.
#define TAB_RUN 16
template <class PL>
__host__ __device__ constexpr uint32_t plan_runs(int pos) { return (PL::entries(pos) - 1 + TAB_RUN - 1) / TAB_RUN; }
template <class PL>
__host__ __device__ constexpr uint32_t plan_runs_total() {
  uint32_t t = 0;
  for (int p = 0; p < PL::P; ++p) t += plan_runs<PL>(p);
  return t;
}
template <class PL>
__global__ void __launch_bounds__(BLOCK) comb_entry_kernel(const ge* __restrict__ bases,
                                                           const uint8_t* __restrict__ dec_ok, uint32_t n_keys,
                                                           uint32_t* __restrict__ tables,
                                                           const uint32_t* __restrict__ slot) {
  constexpr int P = PL::P;
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t per_key = plan_runs_total<PL>();  // runs of entries 1 .. 2^(width-1) over all positions
  if (tid >= per_key * n_keys) return;
  const uint32_t key = (uint32_t)(tid / per_key);
  uint32_t run = (uint32_t)(tid % per_key);
  int pos = 0;
  while (run >= plan_runs<PL>(pos)) run -= plan_runs<PL>(pos++);
  const uint32_t E = PL::entries(pos);
  uint32_t* out = tables + (size_t)(slot ? slot[key] : key) * PL::TABLE_WORDS + (size_t)PL::offset(pos) * 32;
  if (run == 0) {
    niels id;
    niels_identity(id);
    store_niels(out, id);
  }
  const uint32_t j0 = 1 + run * TAB_RUN;
  const uint32_t cnt = min((uint32_t)TAB_RUN, E - j0);
  if (!dec_ok[key]) {
    niels id;
    niels_identity(id);
    for (uint32_t t = 0; t < cnt; ++t) store_niels(out + (size_t)(j0 + t) * 32, id);
    return;
  }
  const ge Q = bases[(size_t)key * P + pos];
  // acc = j0 * Q
  ge acc = Q;
  const int top = 31 - __builtin_clz(j0);
  for (int bb = top - 1; bb >= 0; --bb) {
    ge_dbl(acc, acc);
    if ((j0 >> bb) & 1) { ge t; ge_add(t, acc, Q); acc = t; }
  }
  // the run's points (private arrays: scratch is fine for a one-time build)
  fe X[TAB_RUN], Y[TAB_RUN], Z[TAB_RUN], pre[TAB_RUN];
  for (uint32_t t = 0; t < cnt; ++t) {
    X[t] = acc.X; Y[t] = acc.Y; Z[t] = acc.Z;
    if (t == 0) pre[0] = acc.Z; else fe_mul(pre[t], pre[t - 1], acc.Z);
    if (t + 1 < cnt) { ge nx; ge_add(nx, acc, Q); acc = nx; }
  }
  fe inv;
  fe_invert_gcd(inv, pre[cnt - 1]);
  for (int t = (int)cnt - 1; t >= 0; --t) {
    fe zi;
    if (t > 0) { fe_mul(zi, inv, pre[t - 1]); fe_mul(inv, inv, Z[t]); } else { zi = inv; }
    fe x, y;
    fe_mul(x, X[t], zi);
    fe_mul(y, Y[t], zi);
    niels n;
    niels_from_affine(n, x, y);
    store_niels(out + (size_t)(j0 + t) * 32, n);
  }
}

template <class PL>
static hipError_t build_tables(const uint32_t* d_enc, uint32_t n, int negate, uint32_t* d_tables, uint8_t* d_key_ok,
                               hipStream_t st, const uint32_t* d_slot, uint32_t* d_keys_out, int* wrote) {
  // scratch first: a failed allocation returns before anything the caller's key set holds is touched
  ge* d_bases = nullptr;
  uint8_t* d_dec = nullptr;
  hipError_t e = hipMalloc(&d_bases, sizeof(ge) * (size_t)PL::P * n);
  if (e == hipSuccess) e = hipMalloc(&d_dec, n);
  if (e == hipSuccess) {
    if (wrote) *wrote = 1;
    const uint64_t t1 = (uint64_t)PL::P * n;
    hipLaunchKernelGGL(comb_base_kernel<PL>, dim3((unsigned)((t1 + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, d_enc,
                       n, negate, d_bases, d_dec, d_key_ok, d_slot, d_keys_out);
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    const uint64_t t2 = (uint64_t)plan_runs_total<PL>() * n;
    hipLaunchKernelGGL(comb_entry_kernel<PL>, dim3((unsigned)((t2 + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st,
                       d_bases, d_dec, n, d_tables, d_slot);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  else (void)hipStreamSynchronize(st);  // (nothing may still read the scratch when it is freed)
  if (d_bases) (void)hipFree(d_bases);
  if (d_dec) (void)hipFree(d_dec);
  return e;
}

hipError_t build_comb_tables(int pa, const uint32_t* d_enc, uint32_t n, int negate, uint32_t* d_tables,
                             uint8_t* d_key_ok, hipStream_t st, const uint32_t* d_slot, uint32_t* d_keys_out,
                             int* wrote) {
  if (wrote) *wrote = 0;
  switch (pa) {
    case 0: return build_tables<PLB>(d_enc, n, negate, d_tables, d_key_ok, st, d_slot, d_keys_out, wrote);
    case PLA_HUGE::P: return build_tables<PLA_HUGE>(d_enc, n, negate, d_tables, d_key_ok, st, d_slot, d_keys_out, wrote);
    case PLA_BIG::P: return build_tables<PLA_BIG>(d_enc, n, negate, d_tables, d_key_ok, st, d_slot, d_keys_out, wrote);
    case PLA_MID::P: return build_tables<PLA_MID>(d_enc, n, negate, d_tables, d_key_ok, st, d_slot, d_keys_out, wrote);
    case PLA_SMALL::P: return build_tables<PLA_SMALL>(d_enc, n, negate, d_tables, d_key_ok, st, d_slot, d_keys_out, wrote);
    default: return hipErrorInvalidValue;
  }
}
