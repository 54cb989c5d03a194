// MI355X (gfx950) batch Ed25519 verifier for PBFT prepare/commit quorums:
// kernels + the C ABI declared in include/pbft_verify.h.
//
// Data layout in HBM (one context = one GPU):
//   tabB   comb table of the base point, plan PLB (10 positions of 25/26-bit
//          signed windows, 128-B entries)
//   tabA   one comb table of -A per replica key, same geometry with WA
//   keys   raw 32-byte key encodings (hashed as given) + key_ok bytes
//   batch  SoA: R[N][32], S[N][32], key_idx[N] u16, msg[N][stride]
//   bitmap ceil(N/64) u64 words, one per wavefront (ballot)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/pbft_verify.h"
#include "../../include/pbft_wire.h"
#include "digest_kernels.h"
#include "verify_core.h"

using namespace pbft;

#define PBFT_ENVELOPE_LEN 85
#define BLOCK 256

// Comb plans (verify_core.h `plan`): balanced windows over the 254 bits of a
// signed-digit scalar < 2^253, i.e. the fewest positions (= comb steps) for the
// HBM they take.  Base point: 10 positions (4 x 26 + 6 x 25 bits), 235M entries
// x 128 B = 30 GB, one copy per device shared by all contexts.  Replica keys:
// the widest plan whose tables fit the key-table budget (default 70 % of the
// free HBM, ~180 GB on MI355X; PBFT_OPT_KEY_TABLE_BUDGET_MB): 13 positions
// (7 x 20 + 6 x 19 bits, 671 MB per key: n <= 268), 14 (2 x 19 + 12 x 18,
// 268 MB), 16 (14 x 16 + 2 x 15, 63 MB), else 32 (30 x 8 + 2 x 7, 0.5 MB).
// 23 steps per signature at n = 256.  DESIGN.md §3-4; measured in
// profiles/r01_ab_log.md, profiles/r02_ab_log.md.
#ifndef PBFT_PLAN_B
#define PBFT_PLAN_B 10, 25, 4
#endif
#ifndef PBFT_PLAN_A
#define PBFT_PLAN_A 14, 18, 2
#endif
using PLB = plan<PBFT_PLAN_B>;
using PLA_HUGE = plan<13, 19, 7>;  // 7 x 20 + 6 x 19 bits: 671 MB per key (n = 256: 172 GB)
using PLA_BIG = plan<PBFT_PLAN_A>;
using PLA_MID = plan<16, 15, 14>;
using PLA_SMALL = plan<32, 7, 30>;
static_assert(PLA_HUGE::P < PLA_BIG::P && PLA_BIG::P < PLA_MID::P && PLA_MID::P < PLA_SMALL::P,
              "key plans are told apart by P");

// ------------------------------------------------------------------ errors
static thread_local std::string g_last_error;
static int set_err(int code, const char* what) {
  g_last_error = what;
  return code;
}
#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      char _b[256];                                                                     \
      snprintf(_b, sizeof _b, "%s: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
               __LINE__);                                                               \
      return set_err(PBFT_EHIP, _b);                                                    \
    }                                                                                   \
  } while (0)

// ------------------------------------------------------------------ kernels

// Comb tables for a set of points given by encoding (negate: tables of -P).
// Pass 1, one thread per (key, position): decompress, key_ok, and the
// position's base point 2^bitoff(pos) * (+-P) by bitoff(pos) doublings.
template <class PL>
__global__ void __launch_bounds__(BLOCK) comb_base_kernel(const uint32_t* __restrict__ enc, uint32_t n_keys,
                                                          int negate, ge* __restrict__ bases,
                                                          uint8_t* __restrict__ dec_ok, uint8_t* __restrict__ key_ok) {
  constexpr int P = PL::P;
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (uint64_t)P * n_keys) return;
  const uint32_t key = (uint32_t)(tid / P);
  const int pos = (int)(tid % P);
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = enc[8 * key + i];
  ge A;
  const bool dec = ge_decompress(A, w);
  if (pos == 0) {
    dec_ok[key] = dec ? 1 : 0;
    if (key_ok) key_ok[key] = (dec && !ge_is_small_order(A)) ? 1 : 0;
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
                                                           uint32_t* __restrict__ tables) {
  constexpr int P = PL::P;
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t per_key = plan_runs_total<PL>();  // runs of entries 1 .. 2^(width-1) over all positions
  if (tid >= per_key * n_keys) return;
  const uint32_t key = (uint32_t)(tid / per_key);
  uint32_t run = (uint32_t)(tid % per_key);
  int pos = 0;
  while (run >= plan_runs<PL>(pos)) run -= plan_runs<PL>(pos++);
  const uint32_t E = PL::entries(pos);
  uint32_t* out = tables + (size_t)key * PL::TABLE_WORDS + (size_t)PL::offset(pos) * 32;
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
static int build_tables(const uint32_t* d_enc, uint32_t n, int negate, uint32_t* d_tables, uint8_t* d_key_ok,
                        hipStream_t st) {
  ge* d_bases = nullptr;
  uint8_t* d_dec = nullptr;
  HIP_TRY(hipMalloc(&d_bases, sizeof(ge) * (size_t)PL::P * n));
  HIP_TRY(hipMalloc(&d_dec, n));
  const uint64_t t1 = (uint64_t)PL::P * n;
  hipLaunchKernelGGL(comb_base_kernel<PL>, dim3((unsigned)((t1 + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, d_enc, n,
                     negate, d_bases, d_dec, d_key_ok);
  HIP_TRY(hipGetLastError());
  const uint64_t t2 = (uint64_t)plan_runs_total<PL>() * n;
  hipLaunchKernelGGL(comb_entry_kernel<PL>, dim3((unsigned)((t2 + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, d_bases,
                     d_dec, n, d_tables);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(st));
  HIP_TRY(hipFree(d_bases));
  HIP_TRY(hipFree(d_dec));
  return PBFT_OK;
}

__device__ __forceinline__ void load32(uint32_t w[8], const uint8_t* p) {
  const uint4* q = (const uint4*)p;
  const uint4 a = q[0], b = q[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

// ---- verify, device form ----------------------------------------------------
// Same arithmetic as verify_lane (verify_core.h), split into two kernels by
// register footprint:
//
//  comb_kernel   (one signature per lane, <= 128 VGPRs, 8 KB LDS per wave:
//                 4 waves per SIMD)
//    k = SHA-512(R || A || M) mod L; s < L; signed radix-2^W digits of s and k
//    turned into one table-entry index per comb step (stored [step][Npad] in
//    the HBM workspace, coalesced) plus a 32-bit sign mask held in a VGPR;
//    R' = sum_i T_B[i][s_i] + T_{-A}[i][k_i], every step's 128-B table entry
//    gathered one step AHEAD by line-coalesced LDS-DMA (dma_entry_lines), so
//    the random HBM gathers hide under the previous mixed addition.  Writes
//    R' = (X:Y:Z) limb-major ([limb][N], coalesced) and one flag byte
//    (s < L and key usable).
//  finish_kernel (M = FIN_M signatures per lane, small footprint)
//    Montgomery batch inversion of the M Z's (1 inversion + 3(M-1) muls
//    instead of M inversions), affine x, y, canonical compare with R,
//    small-order test on y, ballot -> one bitmap word per (wave, m).
//
// Step order of the comb: B_0, A_0, B_1, A_1, ... while both scalars have
// positions, then the remaining positions of the longer one.
typedef __attribute__((address_space(3))) void lds_void;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// 16-B LDS read from a 32-bit LDS byte address (ds_read_b128)
__device__ __forceinline__ u32x4 lds_read16(uint32_t addr) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef __attribute__((address_space(3))) const u32x4 lds_u32x4;
  return *(lds_u32x4*)(uintptr_t)addr;
#else
  (void)addr;
  return u32x4{0, 0, 0, 0};
#endif
}
#ifndef FIN_M
#define FIN_M 16
#endif
#ifndef FIN_WAVES_PER_EU
#define FIN_WAVES_PER_EU 1
#endif

template <class PLB_, class PLA_>
struct steps {
  static constexpr int PB = PLB_::P, PA = PLA_::P;
  static constexpr int PMIN = PB < PA ? PB : PA;
  static constexpr int N = PB + PA;
  static_assert(N <= 64, "sign mask holds one bit per step");
  using mask_t = typename std::conditional<(N <= 32), uint32_t, uint64_t>::type;
  // table and position of step j (wave-uniform)
  __host__ __device__ static constexpr bool is_a(int j) { return j < 2 * PMIN ? (j & 1) : (PA > PB); }
  __host__ __device__ static constexpr int pos(int j) { return j < 2 * PMIN ? (j >> 1) : j - PMIN; }
};

// Line-coalesced gather ("transposed" DMA).  A table entry is one 128-B line.
// Lane-per-entry DMA (each lane fetching its own entry in 8 x 16 B) makes
// every wave-instruction touch 64 different lines 16 B at a time, the access
// shape the memory pipeline serves worst (profiles/r01_ab_log.md: the kernel
// ran as fast without its arithmetic).  Here instruction q fetches the 8
// entries of lanes 8q..8q+7 WHOLE: lane L reads 16-B chunk c = (L & 7) ^ (L >> 3)
// of the entry of lane 8q + (L >> 3), so each instruction covers 8 full lines.
// The DMA lands lane L of instruction q at LDS byte 1024 q + 16 L, i.e. entry e
// occupies bytes [128 e, 128 e + 128) with chunk c at position c ^ (e & 7) --
// the XOR swizzle spreads the owner lanes' ds_read_b128 over all banks.
// idx (entry index in 128-B units from `base`) is fetched from its owner lane
// with ds_bpermute (one base address + immediate offsets 32 q).
__device__ __forceinline__ void dma_entry_lines(const uint8_t* base, uint32_t idx, int lane, uint32_t ebuf_lds) {
  const int k = lane >> 3;
  const uint32_t coff = (uint32_t)(((lane & 7) ^ k) << 4);
  const int baddr = k << 2;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint32_t e = (uint32_t)__builtin_amdgcn_ds_bpermute(baddr + 32 * q, (int)idx);
    __builtin_amdgcn_global_load_lds(base + (size_t)e * 128 + coff,
                                     (lds_void*)(uintptr_t)(ebuf_lds + 1024u * q), 16, 0, 0);
  }
}

// 8-B LDS read from a 32-bit LDS byte address (ds_read_b64)
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u32x2 lds_read8(uint32_t addr) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef __attribute__((address_space(3))) const u32x2 lds_u32x2;
  return *(lds_u32x2*)(uintptr_t)addr;
#else
  (void)addr;
  return u32x2{0, 0};
#endif
}

// This lane's entry from its LDS slot (after the DMA landed: vmcnt(0); the ds_reads use integer LDS
// addresses, so the compiler cannot see that they alias the DMA's writes -- hence the explicit wait), as
// (qa, qb, k) for ge_madd_ab: the sign picks hmx/hpx by ADDRESS (entry layout, verify_core.h), so the swap
// costs two XORs instead of 20 masked-select instructions.  Logical byte o of the entry sits at rd0 ^ o
// (dma_entry_lines' chunk swizzle; o < 128, rd0 16-B aligned).
__device__ __forceinline__ void lds_entry_signed(uint32_t rd0, bool neg, fe& qa, fe& qb, fe& k) {
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  asm volatile("" ::: "memory");
  const uint32_t pos = neg ? 0u : 1u;
  const uint32_t a0 = rd0 ^ (pos << 5);          // qa[0..7]: hmx (o = 32) or hpx (o = 0)
  const uint32_t ah = rd0 ^ 64u ^ (pos << 3);    // qa[8..9]: o = 72 or 64
  const u32x4 a_lo = lds_read16(a0), a_hi = lds_read16(a0 ^ 16u);
  const u32x4 b_lo = lds_read16(a0 ^ 32u), b_hi = lds_read16(a0 ^ 48u);
  const u32x2 a_top = lds_read8(ah), b_top = lds_read8(ah ^ 8u);
  const u32x4 k0 = lds_read16(rd0 ^ 80u), k1 = lds_read16(rd0 ^ 96u);
  const u32x2 k2 = lds_read8(rd0 ^ 112u);
  qa.v[0] = a_lo.x; qa.v[1] = a_lo.y; qa.v[2] = a_lo.z; qa.v[3] = a_lo.w;
  qa.v[4] = a_hi.x; qa.v[5] = a_hi.y; qa.v[6] = a_hi.z; qa.v[7] = a_hi.w;
  qa.v[8] = a_top.x; qa.v[9] = a_top.y;
  qb.v[0] = b_lo.x; qb.v[1] = b_lo.y; qb.v[2] = b_lo.z; qb.v[3] = b_lo.w;
  qb.v[4] = b_hi.x; qb.v[5] = b_hi.y; qb.v[6] = b_hi.z; qb.v[7] = b_hi.w;
  qb.v[8] = b_top.x; qb.v[9] = b_top.y;
  k.v[0] = k0.x; k.v[1] = k0.y; k.v[2] = k0.z; k.v[3] = k0.w;
  k.v[4] = k1.x; k.v[5] = k1.y; k.v[6] = k1.z; k.v[7] = k1.w;
  k.v[8] = k2.x; k.v[9] = k2.y;
}

#ifndef PBFT_LAUNDER
#define PBFT_LAUNDER 1
#endif
#ifndef PBFT_COMB_WAVES_PER_EU
#define PBFT_COMB_WAVES_PER_EU 4
#endif
static constexpr uint32_t COMB_LDS_PER_WAVE = 8 * 1024;

template <int LEN, class PLA>
__global__ void __launch_bounds__(BLOCK, PBFT_COMB_WAVES_PER_EU) comb_kernel(
    const uint8_t* __restrict__ R, const uint8_t* __restrict__ S, const uint8_t* __restrict__ key_idx,
    uint32_t rs_stride, uint32_t k_stride,
    const uint8_t* __restrict__ msg, uint32_t msg_len, uint32_t msg_stride, uint64_t N, uint64_t Npad,
    const uint32_t* __restrict__ tabB, const uint32_t* __restrict__ tabA, const uint32_t* __restrict__ keys,
    const uint8_t* __restrict__ key_ok, uint32_t n_keys, uint32_t* __restrict__ xyz, uint8_t* __restrict__ flags,
    uint32_t* __restrict__ eidx, const uint32_t* __restrict__ msg_idx, uint32_t n_msg) {
  using ST = steps<PLB, PLA>;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63;
  // wave-uniform LDS base of this wave's entry buffer (SGPR: the DMA's M0)
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t ebuf = (uint32_t)(uintptr_t)lds + wave * COMB_LDS_PER_WAVE;
  const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;  // < Npad
  const bool live = i < N;
  const uint64_t ii = live ? i : 0;  // dead lanes recompute lane 0 (no OOB reads)
  typename ST::mask_t sgn = 0;        // bit j: digit of step j is negative
  bool s_ok, kok;
  {
    uint32_t r[8], s[8], a[8];
    load32(r, R + (size_t)rs_stride * ii);
    load32(s, S + (size_t)rs_stride * ii);
    uint32_t ki = *(const uint16_t*)(key_idx + (size_t)k_stride * ii);
    kok = ki < n_keys;
    if (!kok) ki = 0;
    kok = kok && key_ok[ki];
    {
      const uint4* kp = (const uint4*)(keys + 8 * ki);
      const uint4 k0 = kp[0], k1 = kp[1];
      a[0] = k0.x; a[1] = k0.y; a[2] = k0.z; a[3] = k0.w; a[4] = k1.x; a[5] = k1.y; a[6] = k1.z; a[7] = k1.w;
    }
    // the signed message: row ii, or the envelope table row msg_idx[ii] (votes form; out of range -> bit 0)
    uint64_t mrow = ii;
    if (msg_idx) {
      mrow = msg_idx[ii];
      kok = kok && mrow < n_msg;
      if (mrow >= n_msg) mrow = 0;
    }
    s_ok = sc_lt_L(s);
    sc_clamp_rejected(s, s_ok);  // s >= L: recode 0, never index past the base-point table
    uint32_t h[16], k[8];
#if PBFT_ABL_NOSHA  // ablation: no challenge hash (k from R and A directly)
#pragma unroll
    for (int t = 0; t < 16; ++t) h[t] = r[t & 7] ^ a[(t + 3) & 7];
#else
    sha512_ram<LEN>(h, r, a, msg + (size_t)msg_stride * mrow, (int)msg_len);
#endif
    sc_reduce512(k, h);
    // per-step entry index (128-B units from the step's table base) and sign
    const uint32_t keybase = ki * PLA::ENTRIES;
    digits ds, dk;
    ds.init(s);
    dk.init(k);
    static_for<ST::N>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      constexpr bool isA = ST::is_a(j);
      constexpr int pos = ST::pos(j);
      int d;
      if constexpr (isA) d = dk.template take_pos<PLA, pos>();
      else d = ds.template take_pos<PLB, pos>();
      const uint32_t ad = (uint32_t)(d < 0 ? -d : d);
      sgn |= (typename ST::mask_t)(d < 0 ? 1u : 0u) << j;
#if PBFT_ABL_FETCH0  // ablation: every lane gathers entry 1 of its position (L2-resident)
      const uint32_t e = (isA ? PLA::offset(pos) : PLB::offset(pos)) + 1u;
#else
      const uint32_t e = isA ? keybase + PLA::offset(pos) + ad : PLB::offset(pos) + ad;
#endif
      eidx[(size_t)j * Npad + i] = e;
    });
  }
  const uint8_t* tB = (const uint8_t*)tabB;
  const uint8_t* tA = (const uint8_t*)tabA;
  const uint32_t rd0 = ebuf + 128u * lane + 16u * (lane & 7);  // logical byte o of my entry at rd0 ^ o
  // (each lane re-reads only the indices it wrote itself: no barrier needed)
  dma_entry_lines(ST::is_a(0) ? tA : tB, eidx[i], lane, ebuf);
  uint32_t nidx = eidx[Npad + i];
  ge P;
  {
    // step 0: P = +-T_B[0][s_0] directly (1 multiplication instead of a 7-multiplication addition)
    fe qa, qb, k;
    const bool neg = (uint32_t)sgn & 1u;
    lds_entry_signed(rd0, neg, qa, qb, k);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): entry in VGPRs before the DMA reuses the buffer
    dma_entry_lines(ST::is_a(1) ? tA : tB, nidx, lane, ebuf);
    nidx = eidx[2 * Npad + i];
    ge_from_ab(P, qa, qb, k, neg);
  }
  for (int j = 1; j < ST::N - 1; ++j) {
    fe qa, qb, k;
    const bool neg = (uint32_t)(sgn >> j) & 1u;
    lds_entry_signed(rd0, neg, qa, qb, k);
    // the entry must be in VGPRs before the DMA overwrites the buffer (WAR on LDS)
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    dma_entry_lines(ST::is_a(j + 1) ? tA : tB, nidx, lane, ebuf);
    if (j + 2 < ST::N) nidx = eidx[(size_t)(j + 2) * Npad + i];
#if PBFT_ABL_NOMADD  // ablation: gathers only, no group arithmetic
#pragma unroll
    for (int t = 0; t < 10; ++t) { P.X.v[t] ^= qa.v[t]; P.Y.v[t] ^= qb.v[t]; P.Z.v[t] += k.v[t] + neg; }
#else
    ge_madd_ab<true>(P, P, qa, qb, k, neg);
#endif
#if PBFT_LAUNDER
    // Keep the loop-carried limbs opaque 32-bit values: otherwise LLVM carries
    // them as the i64 columns they were reduced from and every product with a
    // P limb becomes a 64x32 multiply (2 mads + moves).
#pragma unroll
    for (int t = 0; t < 10; ++t) {
      asm("" : "+v"(P.X.v[t]), "+v"(P.Y.v[t]), "+v"(P.Z.v[t]), "+v"(P.T.v[t]));
    }
#endif
  }
  {
    // last step: R' needs X, Y, Z only (6 multiplications)
    fe qa, qb, k;
    const bool neg = (uint32_t)(sgn >> (ST::N - 1)) & 1u;
    lds_entry_signed(rd0, neg, qa, qb, k);
    ge_madd_ab<false>(P, P, qa, qb, k, neg);
  }
  if (live) {
#pragma unroll
    for (int t = 0; t < 10; ++t) {
      xyz[(size_t)t * N + i] = P.X.v[t];
      xyz[(size_t)(10 + t) * N + i] = P.Y.v[t];
      xyz[(size_t)(20 + t) * N + i] = P.Z.v[t];
    }
    flags[i] = (s_ok && kok) ? 1 : 0;
  }
}

// ---- latency mode: small batches --------------------------------------------
// For small batches (BASELINE config #5: 4096-signature rounds) one lane per
// signature leaves most SIMDs idle, and the round's latency is one lane's
// serial work: SHA-512, 24 comb steps, then the finish kernel's inversion.
// comb_latency_kernel (blocks of 4 waves -- one per SIMD, so each may use the
// whole register file -- and 64 signatures per block) instead
//  * gives every signature SPLIT = 4 lanes: each lane computes the challenge
//    hash itself (it is on the critical path anyway), then the steps
//    j = SPLIT*t + r of the comb (r = lane % SPLIT; lanes without a step in the
//    last round add the identity entry), and the 4 partial points are summed
//    with two shuffle + extended-addition rounds (every lane of the group then
//    holds R');
//  * R' is compressed with ONE divsteps inversion (inv25519.h, ~20 us on the
//    chain) and compared with the canonical R encoding, as the finish kernel
//    does; each wave writes 16 bitmap bits (u16 pieces: piece 4 * block + wave).
// Round 1 instead decompressed R on a fourth wave in parallel (z^((p-5)/8):
// 254 squarings on one wave, ~80 us -- the critical path); PBFT_LAT_DECOMP=1
// keeps that variant for A/B.  ~2.5x lower latency than one lane per signature.
#ifndef PBFT_LAT_DECOMP
#define PBFT_LAT_DECOMP 0
#endif
static constexpr int SPLIT = 4;
static constexpr int LAT_COMB_WAVES = PBFT_LAT_DECOMP ? 3 : 4;
static constexpr int LAT_SIGS = LAT_COMB_WAVES * 64 / 4;  // signatures per block
static constexpr int LAT_BLOCK = 4 * 64;                   // (PBFT_LAT_DECOMP: 3 comb waves + 1 decompression wave)
#ifndef PBFT_SPLIT_BELOW
#define PBFT_SPLIT_BELOW 12288  // measured crossover: 8,192 sigs 0.105 ms here vs 0.133 ms one-lane; 16,384: 0.195 vs 0.133
#endif
static constexpr uint64_t SPLIT_BELOW = PBFT_SPLIT_BELOW;  // batches below this use comb_latency_kernel
static constexpr uint32_t LAT_LDS =
    LAT_COMB_WAVES * COMB_LDS_PER_WAVE + (PBFT_LAT_DECOMP ? 21 * 64 * 4 : 0);  // entry buffers (+ x_R, y_R, ok)

// Line-coalesced gather with per-lane 64-bit entry addresses (the split kernel's
// lanes of one wave gather from both tables in the same step).
__device__ __forceinline__ void dma_entry_lines64(const uint8_t* addr, int lane, uint32_t ebuf_lds) {
  const int k = lane >> 3;
  const uint32_t coff = (uint32_t)(((lane & 7) ^ k) << 4);
  const int baddr = k << 2;
  const uint64_t a = (uint64_t)(uintptr_t)addr;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(baddr + 32 * q, (int)(uint32_t)a);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(baddr + 32 * q, (int)(uint32_t)(a >> 32));
    const uint8_t* src = (const uint8_t*)(uintptr_t)(((uint64_t)hi << 32) | lo);
    __builtin_amdgcn_global_load_lds(src + coff, (lds_void*)(uintptr_t)(ebuf_lds + 1024u * q), 16, 0, 0);
  }
}

FE_FN void fe_shfl_xor(fe& out, const fe& in, int mask) {
#pragma unroll
  for (int t = 0; t < 10; ++t) out.v[t] = (uint32_t)__shfl_xor((int)in.v[t], mask);
}

template <int LEN, class PLA>
__global__ void __launch_bounds__(LAT_BLOCK, 1) comb_latency_kernel(
    const uint8_t* __restrict__ R, const uint8_t* __restrict__ S, const uint8_t* __restrict__ key_idx,
    uint32_t rs_stride, uint32_t k_stride,
    const uint8_t* __restrict__ msg, uint32_t msg_len, uint32_t msg_stride, uint64_t N, uint64_t Lpad,
    const uint32_t* __restrict__ tabB, const uint32_t* __restrict__ tabA, const uint32_t* __restrict__ keys,
    const uint8_t* __restrict__ key_ok, uint32_t n_keys, uint64_t* __restrict__ bitmap,
    const uint8_t** __restrict__ eaddr, const uint32_t* __restrict__ msg_idx, uint32_t n_msg) {
  using ST = steps<PLB, PLA>;
  constexpr int T = (ST::N + SPLIT - 1) / SPLIT;  // local steps per lane
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t ebuf = (uint32_t)(uintptr_t)lds + wave * COMB_LDS_PER_WAVE;
#if PBFT_LAT_DECOMP
  uint32_t* rdec = (uint32_t*)(lds + LAT_COMB_WAVES * COMB_LDS_PER_WAVE);  // [21][64]: x_R, y_R limbs, ok
  if (wave == LAT_COMB_WAVES) {
    // ---- decompression wave: R of signature blockIdx * LAT_SIGS + lane (lanes >= LAT_SIGS idle)
    const uint64_t i = (uint64_t)blockIdx.x * LAT_SIGS + lane;
    const uint64_t ii = i < N ? i : 0;
    uint32_t rr[8], ry[8];
    load32(rr, R + (size_t)rs_stride * ii);
    ge Rp;
#if PBFT_ABL_LAT_NODEC  // ablation: no decompression (timing only)
    bool ok = true;
    fe_zero(Rp.X); fe_zero(Rp.Y);
#else
    bool ok = ge_decompress<true>(Rp, rr);  // dalek 3.2.1 CompressedEdwardsY::decompress (latency-oriented)
#endif
    canon_y(ry, rr);
    ok = ok && !y_is_small_order(ry);  // small-order R (verify_strict)
#pragma unroll
    for (int t = 0; t < 10; ++t) { rdec[t * 64 + lane] = Rp.X.v[t]; rdec[(10 + t) * 64 + lane] = Rp.Y.v[t]; }
    rdec[20 * 64 + lane] = ok ? 1u : 0u;
    __syncthreads();
    return;
  }
#endif
  // ---- comb waves: 16 signatures per wave, SPLIT lanes each
  const uint64_t g = (uint64_t)blockIdx.x * (LAT_COMB_WAVES * 64) + threadIdx.x;  // global comb lane, < Lpad
  const uint64_t i = g / SPLIT;
  const int r = (int)(g % SPLIT);
  const bool live = i < N;
  const uint64_t ii = live ? i : 0;
  uint32_t sgn = 0;  // bit t: digit of local step t is negative
  bool s_ok, kok;
  {
    uint32_t rr[8], s[8], a[8];
    load32(rr, R + (size_t)rs_stride * ii);
    load32(s, S + (size_t)rs_stride * ii);
    uint32_t ki = *(const uint16_t*)(key_idx + (size_t)k_stride * ii);
    kok = ki < n_keys;
    if (!kok) ki = 0;
    kok = kok && key_ok[ki];
    {
      const uint4* kp = (const uint4*)(keys + 8 * ki);
      const uint4 k0 = kp[0], k1 = kp[1];
      a[0] = k0.x; a[1] = k0.y; a[2] = k0.z; a[3] = k0.w; a[4] = k1.x; a[5] = k1.y; a[6] = k1.z; a[7] = k1.w;
    }
    uint64_t mrow = ii;
    if (msg_idx) {
      mrow = msg_idx[ii];
      kok = kok && mrow < n_msg;
      if (mrow >= n_msg) mrow = 0;
    }
    s_ok = sc_lt_L(s);
    sc_clamp_rejected(s, s_ok);  // s >= L: recode 0, never index past the base-point table
    uint32_t h[16], k[8];
    sha512_ram<LEN>(h, rr, a, msg + (size_t)msg_stride * mrow, (int)msg_len);
    sc_reduce512(k, h);
    const uint8_t* tA = (const uint8_t*)tabA + (size_t)ki * PLA::TABLE_WORDS * 4;
    digits ds, dk;
    ds.init(s);
    dk.init(k);
    static_for<SPLIT * T>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      if constexpr (j < ST::N) {
        constexpr bool isA = ST::is_a(j);
        constexpr int pos = ST::pos(j);
        int d;
        if constexpr (isA) d = dk.template take_pos<PLA, pos>();
        else d = ds.template take_pos<PLB, pos>();
        if (j % SPLIT == r) {
          const uint32_t ad = (uint32_t)(d < 0 ? -d : d);
          sgn |= (d < 0 ? 1u : 0u) << (j / SPLIT);
          eaddr[(size_t)(j / SPLIT) * Lpad + g] =
              isA ? tA + ((size_t)PLA::offset(pos) + ad) * 128 : (const uint8_t*)tabB + ((size_t)PLB::offset(pos) + ad) * 128;
        }
      } else if (j % SPLIT == r) {
        eaddr[(size_t)(j / SPLIT) * Lpad + g] = (const uint8_t*)tabB;  // entry 0 of position 0: the identity
      }
    });
  }
  const uint32_t rd0 = ebuf + 128u * lane + 16u * (lane & 7);
  dma_entry_lines64(eaddr[g], lane, ebuf);
  const uint8_t* nadr = eaddr[Lpad + g];
  ge P;
  {
    fe qa, qb, k;
    const bool neg = sgn & 1u;
    lds_entry_signed(rd0, neg, qa, qb, k);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    dma_entry_lines64(nadr, lane, ebuf);
    if (2 < T) nadr = eaddr[2 * Lpad + g];
    ge_from_ab(P, qa, qb, k, neg);
  }
  for (int t = 1; t < T; ++t) {
    fe qa, qb, k;
    const bool neg = (sgn >> t) & 1u;
    lds_entry_signed(rd0, neg, qa, qb, k);
    if (t + 1 < T) {
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      dma_entry_lines64(nadr, lane, ebuf);
      if (t + 2 < T) nadr = eaddr[(size_t)(t + 2) * Lpad + g];
    }
#if !PBFT_ABL_LAT_NOSTEPS  // ablation: gathers only (timing only)
    ge_madd_ab<true>(P, P, qa, qb, k, neg);
#endif
#pragma unroll
    for (int u = 0; u < 10; ++u) asm("" : "+v"(P.X.v[u]), "+v"(P.Y.v[u]), "+v"(P.Z.v[u]), "+v"(P.T.v[u]));
  }
  // sum the SPLIT partial points: lanes r ^ 1, then r ^ 2 (extended addition, complete formulas)
  static_assert(SPLIT == 4, "two combine rounds");
  auto combine = [&](int m) {
    ge Q, Sum;
    fe_shfl_xor(Q.X, P.X, m); fe_shfl_xor(Q.Y, P.Y, m); fe_shfl_xor(Q.Z, P.Z, m); fe_shfl_xor(Q.T, P.T, m);
    ge_add(Sum, P, Q);
    P = Sum;
  };
  combine(1);
  combine(2);
  bool acc = false;
#if PBFT_LAT_DECOMP
  __syncthreads();  // x_R, y_R of the block's signatures are in LDS
  if (r == 0 && live) {
    const int l = (int)(threadIdx.x >> 2);  // signature within the block
    fe xr, yr, t1, t2;
#pragma unroll
    for (int t = 0; t < 10; ++t) { xr.v[t] = rdec[t * 64 + l]; yr.v[t] = rdec[(10 + t) * 64 + l]; }
    fe_mul(t1, xr, P.Z);
    fe_mul(t2, yr, P.Z);
    acc = rdec[20 * 64 + l] && s_ok && kok && fe_eq(P.X, t1) && fe_eq(P.Y, t2);
  }
#else
  {
    // compress R' (one divsteps inversion) and compare with the canonical R encoding (DESIGN.md "R check")
    fe zi, x, y;
    fe_invert_gcd(zi, P.Z);
    fe_mul(x, P.X, zi);
    fe_mul(y, P.Y, zi);
    uint32_t xw[8], yw[8], rr[8], ry[8];
    fe_to_words(xw, x);
    fe_to_words(yw, y);
    load32(rr, R + (size_t)rs_stride * ii);
    canon_y(ry, rr);
    bool eq = (xw[0] & 1u) == (rr[7] >> 31);
#pragma unroll
    for (int t = 0; t < 8; ++t) eq = eq && yw[t] == ry[t];
    acc = r == 0 && live && s_ok && kok && eq && !y_is_small_order(yw);
  }
#endif
  // lanes 4j (j = 0..15) hold this wave's 16 results: one 16-bit piece of the block's bitmap word
  const uint64_t vote = __ballot(acc);
  uint32_t bits = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) bits |= (uint32_t)((vote >> (4 * j)) & 1u) << j;
  const uint64_t piece = (uint64_t)blockIdx.x * LAT_COMB_WAVES + wave;  // signatures 16 piece .. 16 piece + 15
  if (lane == 0 && piece < 4 * ((N + 63) / 64)) ((uint16_t*)bitmap)[piece] = (uint16_t)bits;  // bits past N: 0
}

__device__ __forceinline__ void load_fe(fe& f, const uint32_t* __restrict__ base, uint64_t N, uint64_t i) {
#pragma unroll
  for (int t = 0; t < 10; ++t) f.v[t] = base[(size_t)t * N + i];
}

// Compile-time unrolled helpers (keep the prefix-product array in VGPRs: a
// runtime-indexed array would be placed in scratch, cdna guide §5.4 rule 20).
template <int M>
struct fin_unroll {
  template <class F>
  __device__ static __forceinline__ void up(F&& f) {
    fin_unroll<M - 1>::up(f);
    f(std::integral_constant<int, M - 1>());
  }
  template <class F>
  __device__ static __forceinline__ void down(F&& f) {
    f(std::integral_constant<int, M - 1>());
    fin_unroll<M - 1>::down(f);
  }
};
template <>
struct fin_unroll<0> {
  template <class F>
  __device__ static __forceinline__ void up(F&&) {}
  template <class F>
  __device__ static __forceinline__ void down(F&&) {}
};

// M signatures per lane: lane l of wave w handles i = (w * M + m) * 64 + l.
// M = FIN_M (16) for large rounds; small batches use fewer signatures per lane
// so that more waves share the latency-bound inversion chains (launch_verify).
template <int FM>
__global__ void __launch_bounds__(BLOCK, FIN_WAVES_PER_EU) finish_kernel(const uint8_t* __restrict__ R,
                                                       uint32_t rs_stride,
                                                       const uint32_t* __restrict__ xyz,
                                                       const uint8_t* __restrict__ flags, uint64_t N,
                                                       uint64_t* __restrict__ bitmap) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;
  const uint64_t base = wave * FM * 64 + lane;
  if (wave * FM * 64 >= N) return;
  const uint32_t* Xb = xyz;
  const uint32_t* Yb = xyz + 10 * N;
  const uint32_t* Zb = xyz + 20 * N;
  // prefix products of Z (lanes past N contribute 1)
  fe pre[FM];
  fin_unroll<FM>::up([&](auto mc) {
    constexpr int m = decltype(mc)::value;
    const uint64_t i = base + (uint64_t)m * 64;
    fe z;
    if (i < N) load_fe(z, Zb, N, i); else fe_one(z);
    if constexpr (m == 0) pre[0] = z;
    else fe_mul(pre[m], pre[m - 1], z);
  });
  fe inv;
#if PBFT_FIN_EXP  // A/B: z^(p-2) with latency-oriented carries
  fe_invert<true>(inv, pre[FM - 1]);
#else
  fe_invert_gcd(inv, pre[FM - 1]);  // divsteps: ~19k instructions instead of ~44k on the serial chain
#endif
  fin_unroll<FM>::down([&](auto mc) {
    constexpr int m = decltype(mc)::value;
    const uint64_t i = base + (uint64_t)m * 64;
    const bool live = i < N;
    const uint64_t ii = live ? i : 0;
    fe zi;
    if constexpr (m > 0) {
      fe_mul(zi, inv, pre[m - 1]);   // 1 / Z_m
      fe z;
      if (live) load_fe(z, Zb, N, ii); else fe_one(z);
      fe_mul(inv, inv, z);           // 1 / (Z_0 ... Z_{m-1})
    } else {
      zi = inv;
    }
    fe X, Y, x, y;
    load_fe(X, Xb, N, ii);
    load_fe(Y, Yb, N, ii);
    fe_mul(x, X, zi);
    fe_mul(y, Y, zi);
    uint32_t xw[8], yw[8], r[8], ry[8];
    fe_to_words(xw, x);
    fe_to_words(yw, y);
    load32(r, R + (size_t)rs_stride * ii);
    canon_y(ry, r);
    bool eq = (xw[0] & 1u) == (r[7] >> 31);
#pragma unroll
    for (int t = 0; t < 8; ++t) eq = eq && yw[t] == ry[t];
    const bool ok = live && flags[ii] && eq && !y_is_small_order(yw);
    const uint64_t vote = __ballot(ok);
    if (lane == 0 && live) bitmap[(wave * FM + m)] = vote;
  });
}

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

// Request digests: one byte string per lane (offsets/lens into a packed buffer).
template <int KIND>  // 0 = Blake2b-512, 1 = SHA-256
__global__ void __launch_bounds__(BLOCK) digest_kernel(const uint8_t* __restrict__ data,
                                                       const uint64_t* __restrict__ offsets,
                                                       const uint32_t* __restrict__ lens, uint64_t N,
                                                       uint8_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= N) return;
  const uint8_t* m = data + offsets[i];
  if (KIND == 0) {
    uint8_t d[64];
    blake2b512(d, m, lens[i]);
#pragma unroll
    for (int j = 0; j < 64; ++j) out[64 * i + j] = d[j];
  } else {
    uint8_t d[32];
    sha256(d, m, lens[i]);
#pragma unroll
    for (int j = 0; j < 32; ++j) out[32 * i + j] = d[j];
  }
}

// ------------------------------------------------------------------ context
// A replica key set on one device: raw encodings, key_ok bytes and the -A comb
// tables.  Reference-counted so that contexts cloned for extra streams
// (pbft_verify_ctx_clone) serve batches from the same tables.
struct keyset {
  std::atomic<int> refs{1};
  uint32_t* d_tabA = nullptr;
  uint32_t* d_keys = nullptr;
  uint8_t* d_key_ok = nullptr;
  uint32_t n = 0;
  int pa = 0;  // positions of the key plan (identifies PLA_HUGE / PLA_BIG / PLA_MID / PLA_SMALL)
};
static void keyset_release(keyset* k) {
  if (k && --k->refs == 0) {
    (void)hipFree(k->d_tabA); (void)hipFree(k->d_keys); (void)hipFree(k->d_key_ok);
    delete k;
  }
}

struct pbft_ctx {
  int device = -1;
  hipStream_t stream = nullptr;
  uint32_t* d_tabB = nullptr;
  keyset* ks = nullptr;
  // cached from ks (null / 0 without a key set)
  uint32_t* d_tabA = nullptr;
  uint32_t* d_keys = nullptr;
  uint8_t* d_key_ok = nullptr;
  uint32_t n_keys = 0;
  int pa = 0;  // comb positions of the installed key tables' plan (PLA_HUGE, PLA_BIG, PLA_MID or PLA_SMALL)
  uint64_t split_below = SPLIT_BELOW;  // latency mode below this batch size (env PBFT_SPLIT_BELOW)
  int fin_m = 0;                       // finish-kernel signatures per lane (0 = by batch size)
  uint64_t key_budget_mb = 0;          // key-table budget override (0 = env / default)
  void adopt(keyset* k) {
    keyset_release(ks);
    ks = k;
    d_tabA = k ? k->d_tabA : nullptr; d_keys = k ? k->d_keys : nullptr; d_key_ok = k ? k->d_key_ok : nullptr;
    n_keys = k ? k->n : 0; pa = k ? k->pa : 0;
  }
  // staging for the host-buffer API
  uint8_t* d_stage = nullptr;
  size_t stage_cap = 0;
  uint64_t* d_bitmap = nullptr;
  size_t bitmap_cap = 0;
  // verify workspace: R' limbs [30][N] u32 + flags[N]
  uint8_t* d_work = nullptr;
  size_t work_cap = 0;
  uint64_t work_n = 0;     // signatures the workspace layout is sized for (offsets use this, not the batch N)
  bool work_two = false;   // two xyz/flags halves (pipelined form)
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev_done = nullptr;
  // pipelined device form: comb on the caller's stream, finish on a second stream, two workspace halves
  hipEvent_t ev_comb = nullptr, ev_fin[2] = {nullptr, nullptr};
  bool fin_pending[2] = {false, false};
  int half = 0;
  // host-buffer pipeline: H2D of chunk c+1 (copy stream) overlaps the kernels of chunk c
  hipStream_t cstream = nullptr;
  hipEvent_t ev_copied[2] = {nullptr, nullptr}, ev_consumed[2] = {nullptr, nullptr};
  bool in_flight = false;
  uint64_t* async_out = nullptr;
  uint64_t* h_bitmap = nullptr;  // pinned
  uint64_t async_words = 0;
  float last_ms = 0.f;
};

static int ensure_stage(pbft_ctx* c, size_t bytes, size_t words) {
  if (bytes > c->stage_cap) {
    if (c->d_stage) HIP_TRY(hipFree(c->d_stage));
    c->d_stage = nullptr;
    size_t cap = bytes + (bytes >> 2) + 4096;
    if (hipMalloc(&c->d_stage, cap) != hipSuccess) { c->stage_cap = 0; return set_err(PBFT_ENOMEM, "staging alloc"); }
    c->stage_cap = cap;
  }
  if (words > c->bitmap_cap) {
    if (c->d_bitmap) HIP_TRY(hipFree(c->d_bitmap));
    if (c->h_bitmap) HIP_TRY(hipHostFree(c->h_bitmap));
    c->d_bitmap = nullptr; c->h_bitmap = nullptr;
    size_t cap = words + 64;
    if (hipMalloc(&c->d_bitmap, cap * 8) != hipSuccess) return set_err(PBFT_ENOMEM, "bitmap alloc");
    if (hipHostMalloc(&c->h_bitmap, cap * 8, hipHostMallocDefault) != hipSuccess)
      return set_err(PBFT_ENOMEM, "pinned bitmap alloc");
    c->bitmap_cap = cap;
  }
  return PBFT_OK;
}

// Grow the verify workspace (never inside a stream capture: call
// pbft_verify_reserve first when capturing launches into a graph).
// Workspace per launch of N signatures (Npad = N rounded up to BLOCK):
//   xyz   [30][N] u32   R' limbs, comb -> finish            120 B/sig
//   flags [N] u8                                              1 B/sig
//   eidx  [steps][Npad] u32  per-step table entry indices    4 x steps B/sig
static constexpr int MAX_STEPS = steps<PLB, PLA_SMALL>::N;  // the smallest key plan has the most steps
static_assert(steps<PLB, PLA_SMALL>::N >= steps<PLB, PLA_MID>::N && steps<PLB, PLA_MID>::N >= steps<PLB, PLA_BIG>::N,
              "");
static inline size_t eidx_offset(uint64_t N) { return (121 * (size_t)N + 255) & ~(size_t)255; }
static inline size_t eidx_bytes(uint64_t N) {
  const uint64_t Npad = (N + BLOCK - 1) / BLOCK * BLOCK;
  // (latency mode: SPLIT lanes per signature, 8-byte entry addresses, ceil(steps / SPLIT) per lane)
  const size_t split = 8 * (size_t)((MAX_STEPS + SPLIT - 1) / SPLIT) * (Npad * SPLIT + BLOCK);
  const size_t comb = 4 * (size_t)MAX_STEPS * Npad;
  return ((comb > split ? comb : split) + 255) & ~(size_t)255;
}
// second xyz/flags half (pipelined form) after the entry-index region
static inline size_t half1_offset(uint64_t N) { return eidx_offset(N) + eidx_bytes(N); }
// The layout is a function of c->work_n only, never of the batch at hand: a smaller batch must not move
// the entry-index region onto the xyz/flags half a pipelined finish may still be reading.
static int ensure_work(pbft_ctx* c, uint64_t N, bool two_halves = false) {
  if (N <= c->work_n && (!two_halves || c->work_two)) return PBFT_OK;
  const uint64_t W = N > c->work_n ? N : c->work_n;
  const bool two = two_halves || c->work_two;
  const size_t need = (two ? half1_offset(W) + eidx_offset(W) : half1_offset(W)) + 256;
  // nothing may still read the old workspace: the finishes of earlier pipelined launches, then this stream
  for (int h = 0; h < 2; ++h)
    if (c->fin_pending[h]) { HIP_TRY(hipEventSynchronize(c->ev_fin[h])); c->fin_pending[h] = false; }
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (c->d_work) HIP_TRY(hipDeviceSynchronize());  // a device-form launch may run on a caller's stream
  if (c->d_work) HIP_TRY(hipFree(c->d_work));
  c->d_work = nullptr;
  c->work_cap = 0;
  c->work_n = 0;
  c->work_two = false;
  if (hipMalloc(&c->d_work, need) != hipSuccess) return set_err(PBFT_ENOMEM, "verify workspace alloc");
  c->work_cap = need;
  c->work_n = W;
  c->work_two = two;
  return PBFT_OK;
}

// fst != null: pipelined form -- the finish runs on fst after an event, on one of two
// workspace halves, so the next launch's comb (on st) overlaps it.
static int launch_verify(pbft_ctx* c, const uint8_t* dR, const uint8_t* dS, const uint16_t* dK, const uint8_t* dM,
                         uint32_t msg_len, uint32_t msg_stride, uint64_t N, uint64_t* dB, hipStream_t st,
                         uint32_t rs_stride = 32, uint32_t k_stride = 2, hipStream_t fst = nullptr,
                         const uint32_t* dMI = nullptr, uint32_t n_msg = 0) {
  if (N == 0) return PBFT_OK;
  const uint64_t blocks = (N + BLOCK - 1) / BLOCK;
  if (blocks > 0x7fffffffull) return set_err(PBFT_EINVAL, "N too large for one launch");
  int rc = ensure_work(c, N, fst != nullptr);
  if (rc) return rc;
  int h = 0;
  if (fst) {
    h = c->half;
    c->half ^= 1;
  }
  if (c->fin_pending[h]) HIP_TRY(hipStreamWaitEvent(st, c->ev_fin[h], 0));  // a pipelined finish still reading half h
#if !PBFT_NO_LAUNCH_EVENTS
  HIP_TRY(hipEventRecord(c->ev0, st));
#endif
  const dim3 g((unsigned)blocks), b(BLOCK);
  const uint64_t W = c->work_n;  // layout (>= N)
  uint8_t* hw = c->d_work + (h ? half1_offset(W) : 0);
  uint32_t* xyz = (uint32_t*)hw;
  uint8_t* flags = hw + 120 * N;  // within the half's 121 W bytes
  uint32_t* eidx = (uint32_t*)(c->d_work + eidx_offset(W));
  const uint64_t Npad = blocks * BLOCK;
#define PBFT_LAUNCH_COMB(LEN_, WA_)                                                                               \
  hipLaunchKernelGGL((comb_kernel<LEN_, WA_>), g, b, (BLOCK / 64) * COMB_LDS_PER_WAVE, st, dR, dS,             \
                     (const uint8_t*)dK, rs_stride, k_stride, dM, msg_len, msg_stride, N, Npad, c->d_tabB, c->d_tabA, c->d_keys, c->d_key_ok, c->n_keys, xyz, flags, eidx, dMI, n_msg)
#define PBFT_LAUNCH_SPLIT(LEN_, WA_)                                                                           \
  hipLaunchKernelGGL((comb_latency_kernel<LEN_, WA_>), dim3((unsigned)sblocks), dim3(LAT_BLOCK), LAT_LDS, st, dR, dS, \
                     (const uint8_t*)dK, rs_stride, k_stride, dM, msg_len, msg_stride, N, Lpad, c->d_tabB,           \
                     c->d_tabA, c->d_keys, c->d_key_ok, c->n_keys, dB, (const uint8_t**)eidx, dMI, n_msg)
  const bool latency_mode = N < c->split_below;
  if (latency_mode) {
    // enough blocks for every u16 piece of the ceil(N/64) bitmap words (>= ceil(N / LAT_SIGS))
    const uint64_t pieces = 4 * ((N + 63) / 64);
    const uint64_t sblocks = (pieces + LAT_COMB_WAVES - 1) / LAT_COMB_WAVES, Lpad = sblocks * LAT_COMB_WAVES * 64;
    if (msg_len == PBFT_ENVELOPE_LEN) {
      if (c->pa == PLA_HUGE::P) PBFT_LAUNCH_SPLIT(PBFT_ENVELOPE_LEN, PLA_HUGE);
      else if (c->pa == PLA_BIG::P) PBFT_LAUNCH_SPLIT(PBFT_ENVELOPE_LEN, PLA_BIG);
      else if (c->pa == PLA_MID::P) PBFT_LAUNCH_SPLIT(PBFT_ENVELOPE_LEN, PLA_MID);
      else PBFT_LAUNCH_SPLIT(PBFT_ENVELOPE_LEN, PLA_SMALL);
    } else {
      if (c->pa == PLA_HUGE::P) PBFT_LAUNCH_SPLIT(-1, PLA_HUGE);
      else if (c->pa == PLA_BIG::P) PBFT_LAUNCH_SPLIT(-1, PLA_BIG);
      else if (c->pa == PLA_MID::P) PBFT_LAUNCH_SPLIT(-1, PLA_MID);
      else PBFT_LAUNCH_SPLIT(-1, PLA_SMALL);
    }
  } else if (msg_len == PBFT_ENVELOPE_LEN) {
    if (c->pa == PLA_HUGE::P) PBFT_LAUNCH_COMB(PBFT_ENVELOPE_LEN, PLA_HUGE);
    else if (c->pa == PLA_BIG::P) PBFT_LAUNCH_COMB(PBFT_ENVELOPE_LEN, PLA_BIG);
    else if (c->pa == PLA_MID::P) PBFT_LAUNCH_COMB(PBFT_ENVELOPE_LEN, PLA_MID);
    else PBFT_LAUNCH_COMB(PBFT_ENVELOPE_LEN, PLA_SMALL);
  } else {
    if (c->pa == PLA_HUGE::P) PBFT_LAUNCH_COMB(-1, PLA_HUGE);
    else if (c->pa == PLA_BIG::P) PBFT_LAUNCH_COMB(-1, PLA_BIG);
    else if (c->pa == PLA_MID::P) PBFT_LAUNCH_COMB(-1, PLA_MID);
    else PBFT_LAUNCH_COMB(-1, PLA_SMALL);
  }
#undef PBFT_LAUNCH_COMB
#undef PBFT_LAUNCH_SPLIT
  HIP_TRY(hipGetLastError());
  if (fst) {
#if !PBFT_NO_LAUNCH_EVENTS
    HIP_TRY(hipEventRecord(c->ev1, st));  // pipelined form: last_kernel_ms = the comb (or latency) kernel
#endif
    HIP_TRY(hipEventRecord(c->ev_comb, st));
    HIP_TRY(hipStreamWaitEvent(fst, c->ev_comb, 0));
    st = fst;
  }
  if (!latency_mode) {  // (the latency kernel writes the bitmap itself)
    // signatures per finish lane (one divsteps inversion per lane): measured on MI355X
    // (tools/size_probe.py, profiles/r02_size_probe.md) -- 1 up to 2^16, 4 up to 2^18, then 16
    int fm = N >= ((uint64_t)1 << 19) ? FIN_M : N > ((uint64_t)1 << 16) ? 4 : 1;
    if (c->fin_m) fm = c->fin_m;
#define PBFT_LAUNCH_FIN(M_)                                                                                 \
  hipLaunchKernelGGL(finish_kernel<M_>, dim3((unsigned)((((N + 64 * M_ - 1) / (64 * M_)) * 64 + BLOCK - 1) / \
                                                        BLOCK)),                                           \
                     dim3(BLOCK), 0, st, dR, rs_stride, xyz, flags, N, dB)
    if (fm == FIN_M) PBFT_LAUNCH_FIN(FIN_M);
    else if (fm == 8) PBFT_LAUNCH_FIN(8);
    else if (fm == 4) PBFT_LAUNCH_FIN(4);
    else PBFT_LAUNCH_FIN(1);
#undef PBFT_LAUNCH_FIN
    HIP_TRY(hipGetLastError());
  }
  if (fst) {
    HIP_TRY(hipEventRecord(c->ev_fin[h], fst));
    c->fin_pending[h] = true;
    return PBFT_OK;
  }
#if !PBFT_NO_LAUNCH_EVENTS
  HIP_TRY(hipEventRecord(c->ev1, st));
#endif
  return PBFT_OK;
}

static bool check_batch_args(const void* R, const void* S, const void* K, const void* M, uint32_t msg_len,
                             uint32_t msg_stride, uint64_t N, const void* out) {
  if (N == 0) return out != nullptr || true;
  if (!R || !S || !K || !out) return false;
  if (msg_len > 0 && !M) return false;
  if (msg_stride < msg_len) return false;
  if (msg_len > (1u << 24)) return false;
  return true;
}

// Staging layout of n signatures: R | S | key_idx | msg (+ slack for unaligned message reads).
struct stage_layout {
  size_t offS, offK, offM, bytes;
  stage_layout(uint64_t n, uint32_t msg_stride) {
    offS = 32 * n;
    offK = 64 * n;
    offM = (offK + 2 * n + 255) & ~(size_t)255;
    bytes = (offM + (size_t)msg_stride * n + 64 + 255) & ~(size_t)255;
  }
};

// Host batches above this many signatures are copied and verified in chunks on two
// staging halves: the H2D copy of chunk c+1 (context copy stream) overlaps the
// kernels of chunk c (context stream).  A multiple of 64: chunks own whole
// bitmap words.  2^18 keeps every chunk in the one-lane-per-signature mode.
static constexpr uint64_t PIPE_CHUNK = 1ull << 18;

// Copy a host batch into the staging buffer and launch.  Result: the device bitmap.
static int stage_and_launch(pbft_ctx* c, const uint8_t* R, const uint8_t* S, const uint16_t* K, const uint8_t* M,
                            uint32_t msg_len, uint32_t msg_stride, uint64_t N) {
  const uint64_t words = (N + 63) / 64;
  if (N <= PIPE_CHUNK) {
    const stage_layout L(N, msg_stride);
    int rc = ensure_stage(c, L.bytes, words);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(c->d_stage, R, 32 * N, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_stage + L.offS, S, 32 * N, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_stage + L.offK, K, 2 * N, hipMemcpyHostToDevice, c->stream));
    if ((size_t)msg_stride * N)
      HIP_TRY(hipMemcpyAsync(c->d_stage + L.offM, M, (size_t)msg_stride * N, hipMemcpyHostToDevice, c->stream));
    return launch_verify(c, c->d_stage, c->d_stage + L.offS, (const uint16_t*)(c->d_stage + L.offK),
                         c->d_stage + L.offM, msg_len, msg_stride, N, c->d_bitmap, c->stream);
  }
  const stage_layout L(PIPE_CHUNK, msg_stride);
  int rc = ensure_stage(c, 2 * L.bytes, words);
  if (rc) return rc;
  uint64_t chunk = 0;
  for (uint64_t lo = 0; lo < N; lo += PIPE_CHUNK, ++chunk) {
    const uint64_t n = N - lo < PIPE_CHUNK ? N - lo : PIPE_CHUNK;
    const int b = (int)(chunk & 1);
    uint8_t* base = c->d_stage + (size_t)b * L.bytes;
    if (chunk >= 2) HIP_TRY(hipStreamWaitEvent(c->cstream, c->ev_consumed[b], 0));  // kernels of chunk-2 done
    HIP_TRY(hipMemcpyAsync(base, R + 32 * lo, 32 * n, hipMemcpyHostToDevice, c->cstream));
    HIP_TRY(hipMemcpyAsync(base + L.offS, S + 32 * lo, 32 * n, hipMemcpyHostToDevice, c->cstream));
    HIP_TRY(hipMemcpyAsync(base + L.offK, K + lo, 2 * n, hipMemcpyHostToDevice, c->cstream));
    if ((size_t)msg_stride * n)
      HIP_TRY(hipMemcpyAsync(base + L.offM, M + (size_t)msg_stride * lo, (size_t)msg_stride * n,
                             hipMemcpyHostToDevice, c->cstream));
    HIP_TRY(hipEventRecord(c->ev_copied[b], c->cstream));
    HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_copied[b], 0));
    rc = launch_verify(c, base, base + L.offS, (const uint16_t*)(base + L.offK), base + L.offM, msg_len, msg_stride,
                       n, c->d_bitmap + lo / 64, c->stream);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(c->ev_consumed[b], c->stream));
  }
  return PBFT_OK;
}

// Votes form (include/pbft_verify.h pbft_verify_votes): R, S, key_idx and a 4-byte envelope index per
// signature (70 B instead of 151 B over PCIe) + the batch's table of distinct 85-byte envelopes.
struct votes_layout {
  size_t offS, offK, offI, bytes;
  explicit votes_layout(uint64_t n) {
    offS = 32 * n;
    offK = 64 * n;
    offI = (offK + 2 * n + 15) & ~(size_t)15;
    bytes = (offI + 4 * n + 255) & ~(size_t)255;
  }
};

static int stage_votes_and_launch(pbft_ctx* c, const uint8_t* R, const uint8_t* S, const uint16_t* K,
                                  const uint32_t* IDX, const uint8_t* ENV, uint32_t n_env, uint64_t N) {
  const uint64_t words = (N + 63) / 64;
  const size_t env_bytes = ((size_t)PBFT_ENVELOPE_LEN * n_env + 64 + 255) & ~(size_t)255;  // + read slack
  const uint64_t ch = N < PIPE_CHUNK ? N : PIPE_CHUNK;
  const votes_layout L(ch);
  int rc = ensure_stage(c, env_bytes + (N > PIPE_CHUNK ? 2 : 1) * L.bytes, words);
  if (rc) return rc;
  // envelope table first (copy stream), then each chunk's columns; the kernels of chunk c run on the context
  // stream after its copies, overlapping the copies of chunk c+1
  HIP_TRY(hipMemcpyAsync(c->d_stage, ENV, (size_t)PBFT_ENVELOPE_LEN * n_env, hipMemcpyHostToDevice, c->cstream));
  uint64_t chunk = 0;
  for (uint64_t lo = 0; lo < N; lo += PIPE_CHUNK, ++chunk) {
    const uint64_t n = N - lo < PIPE_CHUNK ? N - lo : PIPE_CHUNK;
    const int b = (int)(chunk & 1);
    uint8_t* base = c->d_stage + env_bytes + (size_t)b * L.bytes;
    if (chunk >= 2) HIP_TRY(hipStreamWaitEvent(c->cstream, c->ev_consumed[b], 0));
    HIP_TRY(hipMemcpyAsync(base, R + 32 * lo, 32 * n, hipMemcpyHostToDevice, c->cstream));
    HIP_TRY(hipMemcpyAsync(base + L.offS, S + 32 * lo, 32 * n, hipMemcpyHostToDevice, c->cstream));
    HIP_TRY(hipMemcpyAsync(base + L.offK, K + lo, 2 * n, hipMemcpyHostToDevice, c->cstream));
    HIP_TRY(hipMemcpyAsync(base + L.offI, IDX + lo, 4 * n, hipMemcpyHostToDevice, c->cstream));
    HIP_TRY(hipEventRecord(c->ev_copied[b], c->cstream));
    HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_copied[b], 0));
    rc = launch_verify(c, base, base + L.offS, (const uint16_t*)(base + L.offK), c->d_stage, PBFT_ENVELOPE_LEN,
                       PBFT_ENVELOPE_LEN, n, c->d_bitmap + lo / 64, c->stream, 32, 2, nullptr,
                       (const uint32_t*)(base + L.offI), n_env);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(c->ev_consumed[b], c->stream));
  }
  return PBFT_OK;
}

// The base-point comb table is a constant of the curve: one copy per device,
// shared by every context on it (reference-counted; 30 GB with the default plan).
static std::mutex g_tabB_mu;
static uint32_t* g_tabB[64] = {};
static int g_tabB_refs[64] = {};

static int acquire_base_table(int device, hipStream_t st, uint32_t** out) {
  std::lock_guard<std::mutex> lk(g_tabB_mu);
  if (device < 0 || device >= 64) return set_err(PBFT_ENODEV, "device ordinal >= 64");
  if (!g_tabB[device]) {
    // base point B = (x, 4/5), x even
    const uint32_t benc[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                              0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
    uint32_t* d_benc = nullptr;
    uint32_t* tab = nullptr;
    HIP_TRY(hipMalloc(&d_benc, 32));
    if (hipMalloc(&tab, PLB::TABLE_WORDS * 4) != hipSuccess) {
      (void)hipFree(d_benc);
      return set_err(PBFT_ENOMEM, "base-point table alloc");
    }
    HIP_TRY(hipMemcpyAsync(d_benc, benc, 32, hipMemcpyHostToDevice, st));
    int rc = build_tables<PLB>(d_benc, 1u, 0, tab, nullptr, st);
    (void)hipFree(d_benc);
    if (rc) { (void)hipFree(tab); return rc; }
    g_tabB[device] = tab;
  }
  ++g_tabB_refs[device];
  *out = g_tabB[device];
  return PBFT_OK;
}

static void release_base_table(int device) {
  std::lock_guard<std::mutex> lk(g_tabB_mu);
  if (device < 0 || device >= 64 || g_tabB_refs[device] == 0) return;
  if (--g_tabB_refs[device] == 0) {
    (void)hipFree(g_tabB[device]);
    g_tabB[device] = nullptr;
  }
}

extern "C" {

const char* pbft_last_error(void) { return g_last_error.c_str(); }

const char* pbft_build_info(void) {
  static char buf[256];
  snprintf(buf, sizeof buf,
           "pbft_verify gfx950 PB=%d PA=%d|%d|%d|%d block=%d entry=128B tabB=%zuB tabA/key=%zuB|%zuB|%zuB|%zuB",
           PLB::P, PLA_HUGE::P, PLA_BIG::P, PLA_MID::P, PLA_SMALL::P, BLOCK, PLB::TABLE_WORDS * 4,
           PLA_HUGE::TABLE_WORDS * 4, PLA_BIG::TABLE_WORDS * 4, PLA_MID::TABLE_WORDS * 4, PLA_SMALL::TABLE_WORDS * 4);
  return buf;
}

int pbft_verify_ctx_create(int device, pbft_ctx** out) {
  if (!out) return set_err(PBFT_EINVAL, "out is null");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return set_err(PBFT_ENODEV, "no HIP device at that ordinal");
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    char b[128];
    snprintf(b, sizeof b, "device %d is %s, this library is built for gfx950", device, prop.gcnArchName);
    return set_err(PBFT_ENODEV, b);
  }
  HIP_TRY(hipSetDevice(device));
  pbft_ctx* c = new pbft_ctx();
  c->device = device;
  HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  if (const char* e = getenv("PBFT_SPLIT_BELOW")) c->split_below = strtoull(e, nullptr, 10);
  HIP_TRY(hipEventCreate(&c->ev0));
  HIP_TRY(hipEventCreate(&c->ev1));
  HIP_TRY(hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming));
  HIP_TRY(hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
  HIP_TRY(hipEventCreateWithFlags(&c->ev_comb, hipEventDisableTiming));
  for (int b = 0; b < 2; ++b) {
    HIP_TRY(hipEventCreateWithFlags(&c->ev_fin[b], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_copied[b], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_consumed[b], hipEventDisableTiming));
  }
  int rc = acquire_base_table(device, c->stream, &c->d_tabB);
  if (rc) {
    (void)hipEventDestroy(c->ev0); (void)hipEventDestroy(c->ev1); (void)hipEventDestroy(c->ev_done);
    for (int b = 0; b < 2; ++b) {
      (void)hipEventDestroy(c->ev_copied[b]); (void)hipEventDestroy(c->ev_consumed[b]); (void)hipEventDestroy(c->ev_fin[b]);
    }
    (void)hipEventDestroy(c->ev_comb);
    (void)hipStreamDestroy(c->cstream);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return rc;
  }
  *out = c;
  return PBFT_OK;
}

int pbft_verify_ctx_destroy(pbft_ctx* c) {
  if (!c) return PBFT_OK;
  // teardown: errors are ignored (nothing useful to report from a destructor)
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  release_base_table(c->device);
  c->adopt(nullptr);
  (void)hipFree(c->d_stage); (void)hipFree(c->d_bitmap); (void)hipFree(c->d_work);
  if (c->h_bitmap) (void)hipHostFree(c->h_bitmap);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->ev_done) (void)hipEventDestroy(c->ev_done);
  for (int b = 0; b < 2; ++b) {
    if (c->fin_pending[b]) (void)hipEventSynchronize(c->ev_fin[b]);
    if (c->ev_copied[b]) (void)hipEventDestroy(c->ev_copied[b]);
    if (c->ev_consumed[b]) (void)hipEventDestroy(c->ev_consumed[b]);
    if (c->ev_fin[b]) (void)hipEventDestroy(c->ev_fin[b]);
  }
  if (c->ev_comb) (void)hipEventDestroy(c->ev_comb);
  if (c->cstream) { (void)hipStreamSynchronize(c->cstream); (void)hipStreamDestroy(c->cstream); }
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return PBFT_OK;
}

int pbft_verify_set_keys(pbft_ctx* c, const uint8_t* A, uint32_t n, uint8_t* key_ok) {
  if (!c || (!A && n)) return set_err(PBFT_EINVAL, "null argument");
  if (n == 0 || n > 65535) return set_err(PBFT_EINVAL, "key count must be 1..65535");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->adopt(nullptr);
  // The widest key window whose tables fit the budget (PBFT_KEY_TABLE_BUDGET_MB, default 96 GiB of the
  // 288 GB HBM) and the free memory: 18-bit (252 MB/key, <= 390 keys by default), 16-bit (67 MB/key), else
  // 8-bit (0.5 MB/key).  Entry indices are 32-bit (n * P * E < 2^32).
  size_t free_b = 0, total_b = 0;
  HIP_TRY(hipMemGetInfo(&free_b, &total_b));
  // default budget: 70 % of the HBM still free (after the 30-GB base-point table: ~180 GB on a 288-GB MI355X)
  size_t budget_mb = free_b / 1048576 * 7 / 10;
  if (const char* e = getenv("PBFT_KEY_TABLE_BUDGET_MB")) budget_mb = strtoull(e, nullptr, 10);
  if (c->key_budget_mb) budget_mb = c->key_budget_mb;
  auto fits = [&](size_t table_words, uint64_t entries_per_key) {
    const size_t bytes = table_words * 4 * (size_t)n;
    return (uint64_t)n * entries_per_key < (1ull << 32) && bytes <= budget_mb * (size_t)1048576 &&
           bytes + ((size_t)4 << 30) < free_b;
  };
  int pa = PLA_SMALL::P;
  size_t tab_words = PLA_SMALL::TABLE_WORDS;
  if (fits(PLA_HUGE::TABLE_WORDS, PLA_HUGE::ENTRIES)) {
    pa = PLA_HUGE::P;
    tab_words = PLA_HUGE::TABLE_WORDS;
  } else if (fits(PLA_BIG::TABLE_WORDS, PLA_BIG::ENTRIES)) {
    pa = PLA_BIG::P;
    tab_words = PLA_BIG::TABLE_WORDS;
  } else if (fits(PLA_MID::TABLE_WORDS, PLA_MID::ENTRIES)) {
    pa = PLA_MID::P;
    tab_words = PLA_MID::TABLE_WORDS;
  }
  const size_t tab_bytes = tab_words * 4 * (size_t)n;
  keyset* k = new keyset();
  k->pa = pa;
  k->n = n;
  if (hipMalloc(&k->d_tabA, tab_bytes) != hipSuccess || hipMalloc(&k->d_keys, 32 * (size_t)n) != hipSuccess ||
      hipMalloc(&k->d_key_ok, n) != hipSuccess) {
    keyset_release(k);
    return set_err(PBFT_ENOMEM, "key table alloc");
  }
  int rc = PBFT_OK;
  if (hipMemcpyAsync(k->d_keys, A, 32 * (size_t)n, hipMemcpyHostToDevice, c->stream) != hipSuccess)
    rc = set_err(PBFT_EHIP, "key upload");
  if (!rc)
    rc = pa == PLA_HUGE::P  ? build_tables<PLA_HUGE>(k->d_keys, n, 1, k->d_tabA, k->d_key_ok, c->stream)
         : pa == PLA_BIG::P ? build_tables<PLA_BIG>(k->d_keys, n, 1, k->d_tabA, k->d_key_ok, c->stream)
         : pa == PLA_MID::P ? build_tables<PLA_MID>(k->d_keys, n, 1, k->d_tabA, k->d_key_ok, c->stream)
                            : build_tables<PLA_SMALL>(k->d_keys, n, 1, k->d_tabA, k->d_key_ok, c->stream);
  if (!rc && key_ok && hipMemcpyAsync(key_ok, k->d_key_ok, n, hipMemcpyDeviceToHost, c->stream) != hipSuccess)
    rc = set_err(PBFT_EHIP, "key_ok download");
  if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = set_err(PBFT_EHIP, "key table build");
  if (rc) {
    keyset_release(k);
    return rc;
  }
  c->adopt(k);
  return PBFT_OK;
}

int pbft_verify_ctx_clone(pbft_ctx* parent, pbft_ctx** out) {
  if (!parent || !out) return set_err(PBFT_EINVAL, "null argument");
  *out = nullptr;
  pbft_ctx* c = nullptr;
  int rc = pbft_verify_ctx_create(parent->device, &c);
  if (rc) return rc;
  if (parent->ks) {
    ++parent->ks->refs;
    c->adopt(parent->ks);
  }
  *out = c;
  return PBFT_OK;
}

int pbft_verify_batch(pbft_ctx* c, const uint8_t* R, const uint8_t* S, const uint16_t* K, const uint8_t* M,
                      uint32_t msg_len, uint32_t msg_stride, uint64_t N, uint64_t* out) {
  int rc = pbft_verify_batch_async(c, R, S, K, M, msg_len, msg_stride, N, out);
  if (rc) return rc;
  return pbft_verify_wait(c);
}

int pbft_verify_batch_async(pbft_ctx* c, const uint8_t* R, const uint8_t* S, const uint16_t* K, const uint8_t* M,
                            uint32_t msg_len, uint32_t msg_stride, uint64_t N, uint64_t* out) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  if (!check_batch_args(R, S, K, M, msg_len, msg_stride, N, out)) return set_err(PBFT_EINVAL, "bad batch arguments");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  if (N == 0) return PBFT_OK;
  HIP_TRY(hipSetDevice(c->device));
  int rc = stage_and_launch(c, R, S, K, M, msg_len, msg_stride, N);
  if (rc) return rc;
  const uint64_t words = (N + 63) / 64;
  HIP_TRY(hipMemcpyAsync(c->h_bitmap, c->d_bitmap, words * 8, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipEventRecord(c->ev_done, c->stream));
  c->in_flight = true;
  c->async_out = out;
  c->async_words = words;
  return PBFT_OK;
}

static int finish_async(pbft_ctx* c) {
  memcpy(c->async_out, c->h_bitmap, c->async_words * 8);
  c->in_flight = false;
  (void)hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1);
  return PBFT_OK;
}

int pbft_verify_poll(pbft_ctx* c) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (!c->in_flight) return 1;
  hipError_t e = hipEventQuery(c->ev_done);
  if (e == hipErrorNotReady) return 0;
  HIP_TRY(e);
  finish_async(c);
  return 1;
}

int pbft_verify_wait(pbft_ctx* c) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (!c->in_flight) return PBFT_OK;
  HIP_TRY(hipEventSynchronize(c->ev_done));
  return finish_async(c);
}

// One host batch over several contexts (GPUs of this process, or cloned contexts
// of one GPU): contiguous 64-aligned shards, one async launch per context, each
// writing its own bitmap words in place (no exchange needed when
// the bitmaps return to one host process).
int pbft_verify_batch_multi(pbft_ctx* const* ctxs, uint32_t n_ctx, const uint8_t* R, const uint8_t* S,
                            const uint16_t* K, const uint8_t* M, uint32_t msg_len, uint32_t msg_stride, uint64_t N,
                            uint64_t* out) {
  if (!ctxs || n_ctx == 0) return set_err(PBFT_EINVAL, "no contexts");
  for (uint32_t i = 0; i < n_ctx; ++i)
    for (uint32_t j = 0; j < i; ++j)
      if (!ctxs[i] || ctxs[i] == ctxs[j]) return set_err(PBFT_EINVAL, "contexts must be distinct and non-null");
  if (!check_batch_args(R, S, K, M, msg_len, msg_stride, N, out)) return set_err(PBFT_EINVAL, "bad batch arguments");
  if (N == 0) return PBFT_OK;
  const uint64_t words = (N + 63) / 64, per = (words + n_ctx - 1) / n_ctx;
  int rc = PBFT_OK;
  uint32_t launched = 0;
  for (; launched < n_ctx; ++launched) {
    const uint64_t lo = launched * per * 64;
    if (lo >= N) break;
    const uint64_t hi = lo + per * 64 < N ? lo + per * 64 : N;
    rc = pbft_verify_batch_async(ctxs[launched], R + 32 * lo, S + 32 * lo, K + lo, M ? M + (size_t)msg_stride * lo : M,
                                 msg_len, msg_stride, hi - lo, out + lo / 64);
    if (rc) break;
  }
  for (uint32_t i = 0; i < launched; ++i) {
    const int w = pbft_verify_wait(ctxs[i]);
    if (!rc) rc = w;
  }
  return rc;
}

int pbft_verify_batch_device(pbft_ctx* c, const uint8_t* dR, const uint8_t* dS, const uint16_t* dK,
                             const uint8_t* dM, uint32_t msg_len, uint32_t msg_stride, uint64_t N, uint64_t* dB,
                             void* stream) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (!check_batch_args(dR, dS, dK, dM, msg_len, msg_stride, N, dB)) return set_err(PBFT_EINVAL, "bad batch arguments");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  return launch_verify(c, dR, dS, dK, dM, msg_len, msg_stride, N, dB, st);
}

int pbft_verify_batch_device_pipelined(pbft_ctx* c, const uint8_t* dR, const uint8_t* dS, const uint16_t* dK,
                                       const uint8_t* dM, uint32_t msg_len, uint32_t msg_stride, uint64_t N,
                                       uint64_t* dB, void* stream, void* finish_stream) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (!stream || !finish_stream || stream == finish_stream)
    return set_err(PBFT_EINVAL, "two distinct non-null streams required");
  if (!check_batch_args(dR, dS, dK, dM, msg_len, msg_stride, N, dB)) return set_err(PBFT_EINVAL, "bad batch arguments");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  HIP_TRY(hipSetDevice(c->device));
  return launch_verify(c, dR, dS, dK, dM, msg_len, msg_stride, N, dB, (hipStream_t)stream, 32, 2,
                       (hipStream_t)finish_stream);
}

int pbft_verify_votes(pbft_ctx* c, const uint8_t* R, const uint8_t* S, const uint16_t* K, const uint32_t* env_idx,
                      const uint8_t* envelopes, uint32_t n_env, uint64_t N, uint64_t* out) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  if (N && (!R || !S || !K || !env_idx || !out || !envelopes || n_env == 0))
    return set_err(PBFT_EINVAL, "bad votes arguments");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  if (N == 0) return PBFT_OK;
  HIP_TRY(hipSetDevice(c->device));
  int rc = stage_votes_and_launch(c, R, S, K, env_idx, envelopes, n_env, N);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->h_bitmap, c->d_bitmap, (N + 63) / 64 * 8, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  memcpy(out, c->h_bitmap, (N + 63) / 64 * 8);
  return PBFT_OK;
}

int pbft_verify_votes_device(pbft_ctx* c, const uint8_t* dR, const uint8_t* dS, const uint16_t* dK,
                             const uint32_t* d_env_idx, const uint8_t* d_envelopes, uint32_t n_env, uint64_t N,
                             uint64_t* dB, void* stream) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (N && (!dR || !dS || !dK || !d_env_idx || !d_envelopes || !dB || n_env == 0))
    return set_err(PBFT_EINVAL, "bad votes arguments");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  return launch_verify(c, dR, dS, dK, d_envelopes, PBFT_ENVELOPE_LEN, PBFT_ENVELOPE_LEN, N, dB, st, 32, 2, nullptr,
                       d_env_idx, n_env);
}

// Binary wire records (include/pbft_wire.h): R at +0, S at +32, envelope at +64,
// key index at +150, stride 160 -- read in place by the same kernels.
int pbft_verify_records_device(pbft_ctx* c, const uint8_t* d_rec, uint64_t N, uint64_t* dB, void* stream) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (N && (!d_rec || !dB)) return set_err(PBFT_EINVAL, "bad batch arguments");
  if (((uintptr_t)d_rec & 15) != 0) return set_err(PBFT_EINVAL, "records must be 16-byte aligned");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  return launch_verify(c, d_rec, d_rec + 32, (const uint16_t*)(d_rec + 150), d_rec + 64, PBFT_ENVELOPE_LEN,
                       PBFT_RECORD_BYTES, N, dB, st, PBFT_RECORD_BYTES, PBFT_RECORD_BYTES);
}

int pbft_verify_records(pbft_ctx* c, const uint8_t* rec, uint64_t N, uint64_t* out) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  if (N && (!rec || !out)) return set_err(PBFT_EINVAL, "bad batch arguments");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  if (N == 0) return PBFT_OK;
  HIP_TRY(hipSetDevice(c->device));
  const uint64_t words = (N + 63) / 64;
  int rc = ensure_stage(c, PBFT_RECORD_BYTES * N + 256, words);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_stage, rec, PBFT_RECORD_BYTES * N, hipMemcpyHostToDevice, c->stream));
  rc = pbft_verify_records_device(c, c->d_stage, N, c->d_bitmap, c->stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out, c->d_bitmap, words * 8, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return PBFT_OK;
}

static int run_digest(pbft_ctx* c, int kind, const uint8_t* data, const uint64_t* offsets, const uint32_t* lens,
                      uint64_t N, uint8_t* out) {
  if (!c || (N && (!offsets || !lens || !out))) return set_err(PBFT_EINVAL, "null argument");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  if (N == 0) return PBFT_OK;
  uint64_t total = 0;
  for (uint64_t i = 0; i < N; ++i) {
    const uint64_t end = offsets[i] + lens[i];
    if (end > total) total = end;
  }
  if (total && !data) return set_err(PBFT_EINVAL, "null data");
  HIP_TRY(hipSetDevice(c->device));
  const size_t outb = (kind == 0 ? 64 : 32) * N;
  const size_t offO = (total + 64 + 255) & ~(size_t)255;
  const size_t offL = offO + ((8 * N + 255) & ~(size_t)255);
  const size_t offOut = offL + ((4 * N + 255) & ~(size_t)255);
  int rc = ensure_stage(c, offOut + outb, 1);
  if (rc) return rc;
  if (total) HIP_TRY(hipMemcpyAsync(c->d_stage, data, total, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_stage + offO, offsets, 8 * N, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_stage + offL, lens, 4 * N, hipMemcpyHostToDevice, c->stream));
  const unsigned blocks = (unsigned)((N + BLOCK - 1) / BLOCK);
  if (kind == 0)
    hipLaunchKernelGGL(digest_kernel<0>, dim3(blocks), dim3(BLOCK), 0, c->stream, c->d_stage,
                       (const uint64_t*)(c->d_stage + offO), (const uint32_t*)(c->d_stage + offL), N,
                       c->d_stage + offOut);
  else
    hipLaunchKernelGGL(digest_kernel<1>, dim3(blocks), dim3(BLOCK), 0, c->stream, c->d_stage,
                       (const uint64_t*)(c->d_stage + offO), (const uint32_t*)(c->d_stage + offL), N,
                       c->d_stage + offOut);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out, c->d_stage + offOut, outb, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return PBFT_OK;
}

int pbft_digest_blake2b512(pbft_ctx* c, const uint8_t* data, const uint64_t* offsets, const uint32_t* lens,
                           uint64_t N, uint8_t* out) {
  return run_digest(c, 0, data, offsets, lens, N, out);
}

int pbft_digest_sha256(pbft_ctx* c, const uint8_t* data, const uint64_t* offsets, const uint32_t* lens, uint64_t N,
                       uint8_t* out) {
  return run_digest(c, 1, data, offsets, lens, N, out);
}

int pbft_sign_batch(pbft_ctx* c, const uint8_t* seeds, uint32_t n_seeds, const uint16_t* seed_idx,
                    const uint8_t* msg, uint32_t msg_len, uint32_t msg_stride, uint64_t N, uint8_t* R, uint8_t* S,
                    uint8_t* pub) {
  if (!c || !seeds || n_seeds == 0 || (N && (!seed_idx || !R || !S)) || (msg_len && !msg) || msg_stride < msg_len)
    return set_err(PBFT_EINVAL, "bad sign arguments");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  for (uint64_t i = 0; i < N; ++i)
    if (seed_idx[i] >= n_seeds) return set_err(PBFT_EINVAL, "seed index out of range");
  HIP_TRY(hipSetDevice(c->device));
  const size_t offI = (32 * (size_t)n_seeds + 255) & ~(size_t)255;
  const size_t offM = offI + ((2 * N + 255) & ~(size_t)255);
  const size_t offR = offM + (((size_t)msg_stride * N + 64 + 255) & ~(size_t)255);
  const size_t offS = offR + 32 * N;
  const size_t offP = offS + 32 * N;
  int rc = ensure_stage(c, offP + 32 * (size_t)n_seeds, 1);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_stage, seeds, 32 * (size_t)n_seeds, hipMemcpyHostToDevice, c->stream));
  if (N) HIP_TRY(hipMemcpyAsync(c->d_stage + offI, seed_idx, 2 * N, hipMemcpyHostToDevice, c->stream));
  if (N && msg_len) HIP_TRY(hipMemcpyAsync(c->d_stage + offM, msg, (size_t)msg_stride * N, hipMemcpyHostToDevice, c->stream));
  uint64_t n_launch = N;
  const uint16_t* d_idx = (const uint16_t*)(c->d_stage + offI);
  std::vector<uint16_t> all;
  if (pub && N == 0) n_launch = 0;
  if (n_launch) {
    const unsigned blocks = (unsigned)((n_launch + BLOCK - 1) / BLOCK);
    if (msg_len == PBFT_ENVELOPE_LEN)
      hipLaunchKernelGGL(sign_kernel<PBFT_ENVELOPE_LEN>, dim3(blocks), dim3(BLOCK), 0, c->stream,
                         (const uint32_t*)c->d_stage, d_idx, c->d_stage + offM, msg_len, msg_stride, n_launch,
                         c->d_tabB, (uint32_t*)(c->d_stage + offR), (uint32_t*)(c->d_stage + offS),
                         pub ? (uint32_t*)(c->d_stage + offP) : nullptr, n_seeds);
    else
      hipLaunchKernelGGL(sign_kernel<-1>, dim3(blocks), dim3(BLOCK), 0, c->stream, (const uint32_t*)c->d_stage,
                         d_idx, c->d_stage + offM, msg_len, msg_stride, n_launch, c->d_tabB,
                         (uint32_t*)(c->d_stage + offR), (uint32_t*)(c->d_stage + offS),
                         pub ? (uint32_t*)(c->d_stage + offP) : nullptr, n_seeds);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(R, c->d_stage + offR, 32 * N, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(S, c->d_stage + offS, 32 * N, hipMemcpyDeviceToHost, c->stream));
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (pub) {
    // public keys of seeds that no lane used are derived by a one-lane-per-seed pass
    std::vector<uint16_t> idx(n_seeds);
    for (uint32_t j = 0; j < n_seeds; ++j) idx[j] = (uint16_t)j;
    uint16_t* d_i2 = nullptr;
    uint32_t *d_r2 = nullptr, *d_s2 = nullptr;
    HIP_TRY(hipMalloc(&d_i2, 2 * (size_t)n_seeds));
    HIP_TRY(hipMalloc(&d_r2, 64 * (size_t)n_seeds));
    d_s2 = d_r2 + 8 * (size_t)n_seeds;
    HIP_TRY(hipMemcpyAsync(d_i2, idx.data(), 2 * (size_t)n_seeds, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(sign_kernel<0>, dim3((n_seeds + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, c->stream,
                       (const uint32_t*)c->d_stage, (const uint16_t*)d_i2, (const uint8_t*)nullptr, 0u, 0u,
                       (uint64_t)n_seeds, c->d_tabB, d_r2, d_s2, (uint32_t*)(c->d_stage + offP), n_seeds);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(pub, c->d_stage + offP, 32 * (size_t)n_seeds, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    (void)hipFree(d_i2);
    (void)hipFree(d_r2);
  }
  return PBFT_OK;
}

int pbft_verify_reserve(pbft_ctx* c, uint64_t max_n) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  HIP_TRY(hipSetDevice(c->device));
  return ensure_work(c, max_n, true);  // both halves: either device form can then be captured
}

int pbft_verify_set_option(pbft_ctx* c, int option, uint64_t value) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  switch (option) {
    case PBFT_OPT_SPLIT_BELOW: c->split_below = value; return PBFT_OK;
    case PBFT_OPT_FINISH_WIDTH:
      if (value != 0 && value != 1 && value != 4 && value != 8 && value != FIN_M)
        return set_err(PBFT_EINVAL, "finish width");
      c->fin_m = (int)value;
      return PBFT_OK;
    case PBFT_OPT_KEY_TABLE_BUDGET_MB: c->key_budget_mb = value; return PBFT_OK;
  }
  return set_err(PBFT_EINVAL, "unknown option");
}

int pbft_verify_ctx_info(pbft_ctx* c, uint32_t* pb, uint32_t* pa, uint32_t* n_keys) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (pb) *pb = (uint32_t)PLB::P;
  if (pa) *pa = (uint32_t)c->pa;
  if (n_keys) *n_keys = c->n_keys;
  return PBFT_OK;
}

float pbft_last_kernel_ms(pbft_ctx* c) {
  if (!c) return -1.f;
  float ms = -1.f;
  if (hipEventSynchronize(c->ev1) != hipSuccess) return -1.f;
  if (hipEventElapsedTime(&ms, c->ev0, c->ev1) != hipSuccess) return -1.f;
  c->last_ms = ms;
  return ms;
}

}  // extern "C"
