// Verify kernels of the MI355X batch verifier (comb_kernel, comb_latency_kernel)
// and their per-plan launchers.  Each key plan's kernels are instantiated in
// their own translation unit (comb_pa13.hip, comb_pa14.hip, comb_pa16.hip,
// comb_pa32.hip) so that the four compile in parallel; pbft_verify.hip holds
// the finish, signing, digest and table kernels and the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

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
#ifndef PBFT_DMA_BATCH
#define PBFT_DMA_BATCH 1
#endif
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
#ifndef PBFT_FIN_LV
#define PBFT_FIN_LV 4  // finish product-tree levels (finish.hip): 4 = one inversion per 16-lane row
                       // (fe_invert_wave<true>), 6 = one per wave (r04 A/B, profiles/r04/ab_fin_lv4.txt: 131k shard
                       // -1.8 %, 2^20 -0.4 %); one depth is compiled, PBFT_OPT_FINISH_TREE selects it or none
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
#ifndef PBFT_DMA_MAD
#define PBFT_DMA_MAD 1
#endif
// 64-bit entry address base + coff + 128 e as ONE v_mad_u64_u32 (LLVM otherwise emits a zero-extending
// v_mov, a v_lshlrev_b64 and a v_lshl_add_u64 per entry: 13.5 vs 4.9 cycles per wave-instruction group)
__device__ __forceinline__ const uint8_t* entry_addr(uint64_t base_coff, uint32_t e) {
#if defined(__HIP_DEVICE_COMPILE__) && PBFT_DMA_MAD
  uint64_t a, cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(a), "=s"(cc) : "v"(e), "s"(128u), "v"(base_coff));
  (void)cc;
  return (const uint8_t*)(uintptr_t)a;
#else
  return (const uint8_t*)(uintptr_t)(base_coff + (uint64_t)e * 128u);
#endif
}
__device__ __forceinline__ void dma_entry_lines(const uint8_t* base, uint32_t idx, int lane, uint32_t ebuf_lds) {
  const int k = lane >> 3;
  const uint32_t coff = (uint32_t)(((lane & 7) ^ k) << 4);
  const int baddr = k << 2;
#if PBFT_DMA_MAD
  uint32_t e[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) e[q] = (uint32_t)__builtin_amdgcn_ds_bpermute(baddr + 32 * q, (int)idx);
  const uint64_t bc = (uint64_t)(uintptr_t)base + coff;
#pragma unroll
  for (int q = 0; q < 8; ++q)
    __builtin_amdgcn_global_load_lds(entry_addr(bc, e[q]), (lds_void*)(uintptr_t)(ebuf_lds + 1024u * q), 16, 0, 0);
#elif PBFT_DMA_BATCH
  // all 8 index fetches first (distinct registers), then the 8 loads: one lgkm wait per step instead of
  // one per load -- the stalls matter where few waves share a SIMD (small shards, latency mode)
  uint32_t e[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) e[q] = (uint32_t)__builtin_amdgcn_ds_bpermute(baddr + 32 * q, (int)idx);
#pragma unroll
  for (int q = 0; q < 8; ++q)
    __builtin_amdgcn_global_load_lds(base + (size_t)e[q] * 128 + coff,
                                     (lds_void*)(uintptr_t)(ebuf_lds + 1024u * q), 16, 0, 0);
#else
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint32_t e = (uint32_t)__builtin_amdgcn_ds_bpermute(baddr + 32 * q, (int)idx);
    __builtin_amdgcn_global_load_lds(base + (size_t)e * 128 + coff,
                                     (lds_void*)(uintptr_t)(ebuf_lds + 1024u * q), 16, 0, 0);
  }
#endif
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

__device__ __forceinline__ void lds_write32(uint32_t addr, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  *(__attribute__((address_space(3))) uint32_t*)(uintptr_t)addr = v;
#else
  (void)addr; (void)v;
#endif
}
__device__ __forceinline__ uint32_t lds_read32(uint32_t addr) {
#if defined(__HIP_DEVICE_COMPILE__)
  return *(__attribute__((address_space(3))) const uint32_t*)(uintptr_t)addr;
#else
  (void)addr;
  return 0;
#endif
}

// the divstep table of fe_invert_tab (inv25519.h), constant-initialised at compile time (40 KB); the kernels
// that invert a wave-uniform value copy it to LDS per block
__device__ const ds_table g_ds_tab;
#include "finish_core.h"

#ifndef PBFT_LAUNDER
#define PBFT_LAUNDER 1
#endif
#ifndef PBFT_COMB_WAVES_PER_EU
#define PBFT_COMB_WAVES_PER_EU 4
#endif
static constexpr uint32_t COMB_LDS_PER_WAVE = 8 * 1024;

// The challenge hash k = SHA-512(R || A || M).  85-byte envelopes: block 2's schedule from the scalar unit
// when the whole wave signs one envelope, else from the votes form's per-envelope table (wk != null), else
// per lane (sha512.h sha512_ram85); other lengths in full.
template <int LEN>
__device__ __forceinline__ void sha512_k(uint32_t h[16], const uint32_t r[8], const uint32_t a[8], const uint8_t* m,
                                         int len, const uint64_t* __restrict__ wk, uint64_t mrow) {
  if constexpr (LEN == PBFT_ENVELOPE_LEN) {
    sha512_ram85(h, r, a, m, wk ? wk + (size_t)SHA_ENV_WORDS * mrow : nullptr);
  } else {
    sha512_ram<LEN>(h, r, a, m, len);
  }
}

// Diagnostic build (PBFT_COMB_STAMPS=1, never the product): every wave of comb_kernel stamps its phases into
// g_comb_stamp (a buffer no other code reads; read back by pbft_debug_comb_stamps in comb_pa13.hip, the 13-position
// plan's translation unit).  Per wave: [0] s_memtime at start, [1] s_memrealtime at start, [2] s_memtime once the
// hash, reduction and digit recoding are done, [3] shader cycles spent in the gathers' vmcnt(0) waits (summed over
// the steps), [4] s_memtime at the end, [5] s_memrealtime at the end, [6] cycles in the steps' lgkmcnt(0) waits,
// [7] the HW_ID register (SE / CU / SIMD of the wave).  VERDICT r04 item 3: attribute the 131k shard's stalls.
#ifndef PBFT_COMB_STAMPS
#define PBFT_COMB_STAMPS 0
#endif
#if PBFT_COMB_STAMPS
#define COMB_STAMP_WAVES 16384
static __device__ uint64_t g_comb_stamp[COMB_STAMP_WAVES][8];
#define COMB_T() __builtin_amdgcn_s_memtime()
#define COMB_RT() __builtin_amdgcn_s_memrealtime()
#endif

// WPB = 8 (PBFT_OPT_COMB_PRIO): blocks of 8 waves, waves w and w ^ 4 of a block on the same SIMD (a workgroup's
// waves go round-robin over the CU's 4 SIMDs), each publishing its step count in LDS.  At every step a wave
// that is ahead of its partner lowers its priority (s_setprio 0) and one that is not raises it (2), so the two
// progress together.  Without it the SIMD issues oldest-first: at 2 waves per SIMD (the 131k shard of an 8-GPU
// round) one wave ran as fast as it runs alone (194k cycles, 105 us) and its partner finished ~55 us later on
// its own, latency-bound (profiles/r05/spread/: lifetimes 193k vs 293k cycles on every SIMD).
static constexpr uint32_t COMB_PRIO_LDS = 64;  // 8 progress words (+ pad) after the 8 entry buffers
template <int LEN, class PLA, bool CHAIN = false, int WPB = 4>
__global__ void __launch_bounds__(64 * WPB, PBFT_COMB_WAVES_PER_EU) comb_kernel(
    const uint8_t* __restrict__ R, const uint8_t* __restrict__ S, const uint8_t* __restrict__ key_idx,
    uint32_t rs_stride, uint32_t k_stride,
    const uint8_t* __restrict__ msg, uint32_t msg_len, uint32_t msg_stride, uint64_t N, uint64_t Npad,
    const uint32_t* __restrict__ tabB, const uint32_t* __restrict__ tabA, const uint32_t* __restrict__ keys,
    const uint8_t* __restrict__ key_ok, uint32_t n_keys, uint32_t* __restrict__ xyz, uint8_t* __restrict__ flags,
    uint32_t* __restrict__ eidx, const uint32_t* __restrict__ msg_idx, uint32_t n_msg, uint32_t mi_stride,
    const uint64_t* __restrict__ wk) {
  using ST = steps<PLB, PLA>;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63;
  // wave-uniform LDS base of this wave's entry buffer (SGPR: the DMA's M0)
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t ebuf = (uint32_t)(uintptr_t)lds + wave * COMB_LDS_PER_WAVE;
  const uint64_t i = (uint64_t)blockIdx.x * (64 * WPB) + threadIdx.x;  // < Npad
  const bool live = i < N;
  const uint64_t ii = live ? i : 0;  // dead lanes recompute lane 0 (no OOB reads)
  typename ST::mask_t sgn = 0;        // bit j: digit of step j is negative
  bool s_ok, kok;
  constexpr bool PRIO = WPB == 8;
  const uint32_t prog = (uint32_t)(uintptr_t)lds + WPB * COMB_LDS_PER_WAVE;  // PRIO: step count per wave
  if constexpr (PRIO) {
    if (lane == 0) lds_write32(prog + 4u * wave, 0u);
    __syncthreads();
  }
#if PBFT_COMB_STAMPS
  const uint64_t st_t0 = COMB_T(), st_rt0 = COMB_RT();
  uint64_t st_wait = 0, st_lgkm = 0, st_hash = 0;
#define COMB_WAIT_VM()                                  \
  do {                                                  \
    const uint64_t a_ = COMB_T();                       \
    __builtin_amdgcn_s_waitcnt(0x0F70);                 \
    st_wait += COMB_T() - a_;                           \
  } while (0)
#define COMB_WAIT_LGKM()                                \
  do {                                                  \
    const uint64_t a_ = COMB_T();                       \
    __builtin_amdgcn_s_waitcnt(0xC07F);                 \
    st_lgkm += COMB_T() - a_;                           \
  } while (0)
#else
#define COMB_WAIT_VM()
#define COMB_WAIT_LGKM() __builtin_amdgcn_s_waitcnt(0xC07F)
#endif
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
      mrow = msg_idx[(size_t)mi_stride * ii];
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
    sha512_k<LEN>(h, r, a, msg + (size_t)msg_stride * mrow, (int)msg_len, wk, mrow);
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
#if PBFT_COMB_STAMPS
  st_hash = COMB_T();
#endif
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
    COMB_WAIT_VM();
    lds_entry_signed(rd0, neg, qa, qb, k);
    COMB_WAIT_LGKM();  // lgkmcnt(0): entry in VGPRs before the DMA reuses the buffer
    dma_entry_lines(ST::is_a(1) ? tA : tB, nidx, lane, ebuf);
    nidx = eidx[2 * Npad + i];
    ge_from_ab(P, qa, qb, k, neg);
  }
  for (int j = 1; j < ST::N - 1; ++j) {
    fe qa, qb, k;
    const bool neg = (uint32_t)(sgn >> j) & 1u;
    uint32_t partner = 0;
    if constexpr (PRIO) {
      if (lane == 0) lds_write32(prog + 4u * wave, (uint32_t)j);
      partner = lds_read32(prog + 4u * (wave ^ 4u));
    }
    COMB_WAIT_VM();
    lds_entry_signed(rd0, neg, qa, qb, k);
    // the entry must be in VGPRs before the DMA overwrites the buffer (WAR on LDS)
    COMB_WAIT_LGKM();  // lgkmcnt(0)
    if constexpr (PRIO) {
      if ((uint32_t)j > (uint32_t)__builtin_amdgcn_readfirstlane((int)partner)) __builtin_amdgcn_s_setprio(0);
      else __builtin_amdgcn_s_setprio(2);
    }
    dma_entry_lines(ST::is_a(j + 1) ? tA : tB, nidx, lane, ebuf);
    if (j + 2 < ST::N) nidx = eidx[(size_t)(j + 2) * Npad + i];
#if PBFT_ABL_NOMADD  // ablation: gathers only, no group arithmetic
#pragma unroll
    for (int t = 0; t < 10; ++t) { P.X.v[t] ^= qa.v[t]; P.Y.v[t] ^= qb.v[t]; P.Z.v[t] += k.v[t] + neg; }
#else
    ge_madd_ab<true, CHAIN>(P, P, qa, qb, k, neg);
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
    COMB_WAIT_VM();
    lds_entry_signed(rd0, neg, qa, qb, k);
    if constexpr (PRIO) {
      if (lane == 0) lds_write32(prog + 4u * wave, 0xFFFFu);  // done: the partner is never "ahead" of me
    }
    ge_madd_ab<false, CHAIN>(P, P, qa, qb, k, neg);
  }
#if PBFT_COMB_STAMPS
  {
    const uint64_t t_end = COMB_T(), rt_end = COMB_RT();
    const uint64_t gw = (uint64_t)blockIdx.x * WPB + wave;
    if (lane == 0 && gw < COMB_STAMP_WAVES) {
      uint64_t* o = g_comb_stamp[gw];
      o[0] = st_t0; o[1] = st_rt0; o[2] = st_hash; o[3] = st_wait; o[4] = t_end; o[5] = rt_end; o[6] = st_lgkm;
      o[7] = (uint64_t)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)) |       // HW_ID (hwreg 4)
             ((uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11)) << 32);  // XCC_ID (hwreg 20)
    }
  }
#endif
#undef COMB_WAIT_VM
#undef COMB_WAIT_LGKM
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

// ---- pair mode: two waves per 64 signatures (mid-size batches) -----------------
// Below ~2^18 signatures comb_kernel has fewer than 4 waves per SIMD in one generation (2^17: 2,048 waves, 2 per
// SIMD; 2^16: 1 per SIMD), so the VALU idles in every stall another wave would fill (VALUBusy 72.7 % at 2^17
// against 92 % at 2^20).  comb_pair_kernel splits each signature's sum over two waves of one block:
//  * role 0 (the hashing wave): R, A, M -> k = SHA-512(R || A || M) mod L, the entry indices of all PA key-table
//    positions (eidx rows PB..PB+PA-1) and their signs (LDS), then the sum of key positions 0..A0-1;
//  * role 1: s -> the PB base-point positions, then key positions A0..PA-1 once role 0 has published them
//    (one block barrier, placed so that it precedes the first read of a key-position index);
//  * role 1 leaves its extended point in LDS (its own entry buffer + the pair's 2 KB), a second barrier, and
//    role 0 adds it (one 8-multiplication extended addition, complete) and writes X, Y, Z for finish_kernel.
// A0 balances the two waves' VALU (SHA-512 + reduction ~ 6 mixed additions).  Twice the waves for the same work
// plus one addition per signature; the same R' = [s]B - [k]A, so the finish and the bitmap are unchanged.
// Measured (profiles/r04/pair/): 2^15 signatures -29 %, 2^16 -8 %, 2^17 even (VALUBusy 72.7 -> 76 %: the waves
// of one generation start and stall together, and the combining addition adds ~4 % VALU), 2^18 +2 %; so by batch
// size up to PBFT_PAIR_MAX_N.  Both roles run one copy of the step loop: with a loop per role the instruction
// footprint of SHA-512 + two loops made the kernel 5 % slower at 2^17.
#ifndef PBFT_PAIR_MIN_N
#define PBFT_PAIR_MIN_N 0u  // (below the latency kernel's threshold no batch reaches the one-lane kernels)
#endif
#ifndef PBFT_PAIR_MAX_N
#define PBFT_PAIR_MAX_N (3u << 15)  // by batch size: faster up to 2^16 (-29 % at 2^15, -8 % at 2^16), even at 2^17
                                    // (profiles/r04/pair/)
#endif
static constexpr uint32_t PAIR_SIGS = BLOCK / 2;     // signatures per block
static constexpr uint32_t PAIR_XLDS = 8 * 64 * 4;     // per pair: limbs 32..39 of the exchanged point / sign words
static constexpr size_t PAIR_LDS = (BLOCK / 64) * COMB_LDS_PER_WAVE + (BLOCK / 128) * PAIR_XLDS;
#ifndef PBFT_PAIR_A0_ADJ
#define PBFT_PAIR_A0_ADJ 0  // key positions of role 0: (PB + PA - 6) / 2 + this
#endif
#ifndef PBFT_PAIR_BAR
#define PBFT_PAIR_BAR 0  // role 1's step at which it waits for role 0's indices (0: PB - 2, the latest possible)
#endif
#ifndef PBFT_PAIR_FLIP
#define PBFT_PAIR_FLIP 0  // 1: the wave -> role map flips with the parity of blockIdx (roles mixed over SIMDs)
#endif
template <class PLA>
struct pair_split {
  static constexpr int PB = PLB::P, PA = PLA::P;
  static constexpr int A0r = (PB + PA - 6) / 2 + PBFT_PAIR_A0_ADJ;
  static constexpr int BAR = PBFT_PAIR_BAR ? PBFT_PAIR_BAR : PB - 2;
  static constexpr int A0 = A0r < 1 ? 1 : A0r > PA - 1 ? PA - 1 : A0r;  // key positions of role 0
  static constexpr int N1 = PB + PA - A0;                                  // steps of role 1
  static_assert(BAR >= 1 && BAR <= PB - 2 && N1 <= 32, "role 1 waits before its first key-position index read; "
                "its sign mask is 32 bits");
};

template <int LEN, class PLA>
__global__ void __launch_bounds__(BLOCK, PBFT_COMB_WAVES_PER_EU) comb_pair_kernel(
    const uint8_t* __restrict__ R, const uint8_t* __restrict__ S, const uint8_t* __restrict__ key_idx,
    uint32_t rs_stride, uint32_t k_stride,
    const uint8_t* __restrict__ msg, uint32_t msg_len, uint32_t msg_stride, uint64_t N, uint64_t Npad,
    const uint32_t* __restrict__ tabB, const uint32_t* __restrict__ tabA, const uint32_t* __restrict__ keys,
    const uint8_t* __restrict__ key_ok, uint32_t n_keys, uint32_t* __restrict__ xyz, uint8_t* __restrict__ flags,
    uint32_t* __restrict__ eidx, const uint32_t* __restrict__ msg_idx, uint32_t n_msg, uint32_t mi_stride,
    const uint64_t* __restrict__ wk) {
  using SP = pair_split<PLA>;
  constexpr int PB = SP::PB, PA = SP::PA, A0 = SP::A0, N1 = SP::N1;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t flip = PBFT_PAIR_FLIP ? (uint32_t)__builtin_popcount(blockIdx.x) & 1u : 0u;
  const uint32_t pair = wave >> 1, role = (wave & 1) ^ flip;
  const uint32_t lds0 = (uint32_t)(uintptr_t)lds;
  const uint32_t ebuf = lds0 + wave * COMB_LDS_PER_WAVE;
  const uint32_t pbuf = lds0 + (2 * pair + (1 ^ flip)) * COMB_LDS_PER_WAVE;        // role 1's point, limbs 0..31
  const uint32_t xbuf = lds0 + (BLOCK / 64) * COMB_LDS_PER_WAVE + pair * PAIR_XLDS;  // limbs 32..39; sign words
  const uint64_t i = (uint64_t)blockIdx.x * PAIR_SIGS + pair * 64 + lane;  // < Npad
  const bool live = i < N;
  const uint64_t ii = live ? i : 0;
  const uint8_t* tB = (const uint8_t*)tabB;
  const uint8_t* tA = (const uint8_t*)tabA;
  const uint32_t rd0 = ebuf + 128u * lane + 16u * (lane & 7);
  uint32_t* const erow = eidx + i;  // step row r at erow[r * Npad]
  ge P;
  uint32_t sgn = 0;  // bit t: digit of this role's step t is negative
  bool s_ok = false;  // role 1
  if (role == 0) {
    bool kok;
    {
      uint32_t r[8], a[8];
      load32(r, R + (size_t)rs_stride * ii);
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
        mrow = msg_idx[(size_t)mi_stride * ii];
        kok = kok && mrow < n_msg;
        if (mrow >= n_msg) mrow = 0;
      }
      uint32_t h[16], k[8];
      sha512_k<LEN>(h, r, a, msg + (size_t)msg_stride * mrow, (int)msg_len, wk, mrow);
      sc_reduce512(k, h);
      const uint32_t keybase = ki * PLA::ENTRIES;
      digits dk;
      dk.init(k);
      static_for<PA>([&](auto pc) {
        constexpr int pos = decltype(pc)::value;
        const int d = dk.template take_pos<PLA, pos>();
        sgn |= (d < 0 ? 1u : 0u) << pos;
        erow[(size_t)(PB + pos) * Npad] = keybase + PLA::offset(pos) + (uint32_t)(d < 0 ? -d : d);
      });
    }
    // key positions A0.. and the key's usability for role 1
    lds_write32(xbuf + 4u * lane, (sgn >> A0) | (kok ? 0x80000000u : 0u));
    __syncthreads();  // (1) role 1 may read key-position indices from here on
  } else {
    uint32_t s[8];
    load32(s, S + (size_t)rs_stride * ii);
    s_ok = sc_lt_L(s);
    sc_clamp_rejected(s, s_ok);
    digits ds;
    ds.init(s);
    static_for<PB>([&](auto pc) {
      constexpr int pos = decltype(pc)::value;
      const int d = ds.template take_pos<PLB, pos>();
      sgn |= (d < 0 ? 1u : 0u) << pos;
      erow[(size_t)pos * Npad] = PLB::offset(pos) + (uint32_t)(d < 0 ? -d : d);
    });
  }
  // Both roles run the SAME step loop (one copy of its ~9 KB of code in the instruction cache while the other
  // role hashes).  Step t of a role: table tB for t < nb, else tA; eidx row t + (t < nb ? 0 : roff).
  //   role 0: nb = 0,  roff = PB       (key positions 0 .. A0-1), NS = A0
  //   role 1: nb = PB, roff = A0       (base-point positions, then key positions A0 .. PA-1), NS = N1
  // role 1 meets barrier (1) at step bar, before its first read of a key-position index.
  const int nb = role ? PB : 0, roff = role ? A0 : PB, NS = role ? N1 : A0, bar = role ? SP::BAR : -1;
  auto tab = [&](int t) { return t < nb ? tB : tA; };
  auto row = [&](int t) { return (size_t)(t < nb ? t : t + roff) * Npad; };
  dma_entry_lines(tab(0), erow[row(0)], lane, ebuf);
  uint32_t nidx = NS > 1 ? erow[row(1)] : 0u;
  {
    fe qa, qb, k;
    const bool neg = sgn & 1u;
    lds_entry_signed(rd0, neg, qa, qb, k);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if (NS > 1) dma_entry_lines(tab(1), nidx, lane, ebuf);
    if (NS > 2) nidx = erow[row(2)];
    ge_from_ab(P, qa, qb, k, neg);
  }
  for (int t = 1; t < NS; ++t) {
    if (t == bar) {
      __syncthreads();  // (1): the key positions' indices and signs are published
      const uint32_t w = lds_read32(xbuf + 4u * lane);
      sgn |= (w & 0x7fffffffu) << PB;
      if (live) flags[i] = (s_ok && (w >> 31)) ? 1 : 0;
    }
    fe qa, qb, k;
    const bool neg = (sgn >> t) & 1u;
    lds_entry_signed(rd0, neg, qa, qb, k);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if (t + 1 < NS) dma_entry_lines(tab(t + 1), nidx, lane, ebuf);
    if (t + 2 < NS) nidx = erow[row(t + 2)];
    ge_madd_ab<true, true>(P, P, qa, qb, k, neg);
#pragma unroll
    for (int q = 0; q < 10; ++q) asm("" : "+v"(P.X.v[q]), "+v"(P.Y.v[q]), "+v"(P.Z.v[q]), "+v"(P.T.v[q]));
  }
  if (role) {
    // the point to role 0: limb-major (conflict-free), X Y Z T[0..1] in this wave's entry buffer (its last entry
    // has been read: LDS operations of one wave complete in order), T[2..9] in the pair's area (its sign words
    // were read at barrier 1)
#pragma unroll
    for (int q = 0; q < 10; ++q) {
      const uint32_t o = 4u * (64u * q + lane);
      lds_write32(pbuf + o, P.X.v[q]);
      lds_write32(pbuf + 64u * 4u * 10u + o, P.Y.v[q]);
      lds_write32(pbuf + 64u * 4u * 20u + o, P.Z.v[q]);
      if (q < 2) lds_write32(pbuf + 64u * 4u * 30u + o, P.T.v[q]);
      else lds_write32(xbuf + 4u * (64u * (q - 2) + lane), P.T.v[q]);
    }
    __syncthreads();  // (2)
    return;
  }
  __syncthreads();  // (2) role 1's point is in LDS
  // R' = P + Q (ge_add's arithmetic without T3; Q's coordinates read from LDS as they are needed)
  auto lds_fe = [&](fe& f, int c) {
#pragma unroll
    for (int q = 0; q < 10; ++q) {
      const int l = 10 * c + q;
      f.v[q] = l < 32 ? lds_read32(pbuf + 4u * (64u * l + lane)) : lds_read32(xbuf + 4u * (64u * (l - 32) + lane));
    }
  };
  auto mul1 = [](fe& h, const fe& f, const fe& g) {
    fe* const ho[1] = {&h};
    const fe* const fo[1] = {&f};
    const fe* const go[1] = {&g};
    fe_mul_chain<1>(ho, fo, go);
  };
  fe a, b, c, t, u, w;
  lds_fe(u, 1);
  lds_fe(w, 0);
  fe_sub(t, P.Y, P.X); fe_carry(t);
  fe_sub(a, u, w); fe_carry(a);
  mul1(a, t, a);                        // A = (Y1 - X1)(Y2 - X2)
  fe_add(t, P.Y, P.X);
  fe_add(b, u, w);
  mul1(b, t, b);                        // B = (Y1 + X1)(Y2 + X2)
  lds_fe(u, 3);
  mul1(c, P.T, u);
  fe_const_2d(w);
  mul1(c, c, w);                        // C = 2d T1 T2
  lds_fe(u, 2);
  mul1(t, P.Z, u);
  fe_add(t, t, t);                      // D = 2 Z1 Z2
  fe e, f, g, h;
  fe_sub(e, b, a); fe_sub(f, t, c); fe_add(g, t, c); fe_add(h, b, a);
  fe_carry(e); fe_carry(f); fe_carry(g); fe_carry(h);
  fe X3, Y3, Z3;
  {
    fe* const ho[3] = {&X3, &Y3, &Z3};
    const fe* const fo[3] = {&e, &g, &f};
    const fe* const go[3] = {&f, &h, &g};
    fe_mul_chain<3>(ho, fo, go);
  }
  if (live) {
#pragma unroll
    for (int q = 0; q < 10; ++q) {
      xyz[(size_t)q * N + i] = X3.v[q];
      xyz[(size_t)(10 + q) * N + i] = Y3.v[q];
      xyz[(size_t)(20 + q) * N + i] = Z3.v[q];
    }
  }
}

// ---- latency mode: small batches --------------------------------------------
// For small batches (BASELINE config #5: 4096-signature rounds) one lane per
// signature leaves most SIMDs idle, and the round's latency is one lane's
// serial work: SHA-512, 24 comb steps, then the finish kernel's inversion.
// comb_latency_kernel (blocks of 4 waves -- one per SIMD, so each may use the
// whole register file -- and 64 signatures per block) instead
//  * gives every signature SPLIT = 4 (or 8) lanes: each lane computes the challenge
//    hash itself (it is on the critical path anyway), then the steps
//    j = SPLIT*t + r of the comb (r = lane % SPLIT; lanes without a step in the
//    last round add the identity entry), and the SPLIT partial points are summed
//    with log2(SPLIT) shuffle + extended-addition rounds (every lane of the group
//    then holds R');
//  * R' is compressed with ONE inversion per wave (product tree over the wave's
//    signatures + variable-time divsteps, inv25519.h) and compared with the
//    canonical R encoding, as the finish kernel does; each wave writes its
//    64 / SPLIT bitmap bits (piece SPLIT-dependent u16 / u8).
// Round 1 instead decompressed R on a fourth wave in parallel (z^((p-5)/8):
// 254 squarings on one wave, ~80 us -- the critical path); PBFT_LAT_DECOMP=1
// keeps that variant for A/B.  ~2.5x lower latency than one lane per signature.
#ifndef PBFT_LAT_DECOMP
#define PBFT_LAT_DECOMP 0
#endif
#ifndef PBFT_LAT_TREE
#define PBFT_LAT_TREE 1  // one variable-time inversion per wave (cross-lane product tree)
#endif
// Lanes per signature: 8 up to PBFT_LAT_WIDE_UPTO signatures (3 comb steps per lane, 3 combine rounds), 4
// above (the 8-lane grid would exceed one wave per SIMD): 1k 0.0900 -> 0.0861 ms, 4k 0.0919 -> 0.0885, 8k
// 0.0932 -> 0.0920, 12k 0.0961 -> 0.1280 (profiles/r02_ab_log.md).
#ifndef PBFT_LAT_WIDE_UPTO
#define PBFT_LAT_WIDE_UPTO 8192
#endif
static constexpr uint64_t LAT_WIDE_UPTO = PBFT_LAT_WIDE_UPTO;
static constexpr int LAT_COMB_WAVES = PBFT_LAT_DECOMP ? 3 : 4;
#ifndef PBFT_LAT_TAB
#define PBFT_LAT_TAB (PBFT_LAT_TREE && !PBFT_LAT_DECOMP)  // table-driven divsteps for the wave's inversion
#endif
#ifndef PBFT_LAT_ROWS
#define PBFT_LAT_ROWS 1  // the product tree per 16-lane row, four inversions per wave (fe_invert_wave<true>);
                         // 0: per wave (r04 A/B, profiles/r04/ab_lat_rows.txt: 4k p50 -1.6 %, 8k -2.0 %)
#endif
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
#if PBFT_DMA_BATCH
  uint32_t lo[8], hi[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    lo[q] = (uint32_t)__builtin_amdgcn_ds_bpermute(baddr + 32 * q, (int)(uint32_t)a);
    hi[q] = (uint32_t)__builtin_amdgcn_ds_bpermute(baddr + 32 * q, (int)(uint32_t)(a >> 32));
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint8_t* src = (const uint8_t*)(uintptr_t)(((uint64_t)hi[q] << 32) | lo[q]);
    __builtin_amdgcn_global_load_lds(src + coff, (lds_void*)(uintptr_t)(ebuf_lds + 1024u * q), 16, 0, 0);
  }
#else
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(baddr + 32 * q, (int)(uint32_t)a);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(baddr + 32 * q, (int)(uint32_t)(a >> 32));
    const uint8_t* src = (const uint8_t*)(uintptr_t)(((uint64_t)hi << 32) | lo);
    __builtin_amdgcn_global_load_lds(src + coff, (lds_void*)(uintptr_t)(ebuf_lds + 1024u * q), 16, 0, 0);
  }
#endif
}

FE_FN void fe_shfl_xor(fe& out, const fe& in, int mask) {
#pragma unroll
  for (int t = 0; t < 10; ++t) out.v[t] = (uint32_t)__shfl_xor((int)in.v[t], mask);
}

template <int LEN, class PLA, int SPLIT>
__global__ void __launch_bounds__(LAT_BLOCK, 1) comb_latency_kernel(
    const uint8_t* __restrict__ R, const uint8_t* __restrict__ S, const uint8_t* __restrict__ key_idx,
    uint32_t rs_stride, uint32_t k_stride,
    const uint8_t* __restrict__ msg, uint32_t msg_len, uint32_t msg_stride, uint64_t N, uint64_t Lpad,
    const uint32_t* __restrict__ tabB, const uint32_t* __restrict__ tabA, const uint32_t* __restrict__ keys,
    const uint8_t* __restrict__ key_ok, uint32_t n_keys, uint64_t* __restrict__ bitmap,
    const uint8_t** __restrict__ eaddr, const uint32_t* __restrict__ msg_idx, uint32_t n_msg, uint32_t mi_stride,
    const uint64_t* __restrict__ wk) {
  static_assert(SPLIT == 4 || SPLIT == 8, "2 or 3 combine rounds");
  static_assert(!PBFT_LAT_DECOMP || SPLIT == 4, "the decompression-wave variant pairs 4 lanes per signature");
  constexpr int LAT_SW = 64 / SPLIT;                 // signatures per wave (bits of a wave's bitmap piece)
  constexpr int LAT_SIGS = LAT_COMB_WAVES * LAT_SW;  // signatures per block
  (void)LAT_SIGS;
  using ST = steps<PLB, PLA>;
  constexpr int T = (ST::N + SPLIT - 1) / SPLIT;  // local steps per lane
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t ebuf = (uint32_t)(uintptr_t)lds + wave * COMB_LDS_PER_WAVE;
#if PBFT_LAT_TAB && !PBFT_ABL_NOINV
  // divstep table for the wave's one inversion (inv25519.h fe_invert_tab): every thread copies its share now,
  // the barrier before the inversion publishes it (every wave of the block reaches that barrier)
  __shared__ uint64_t ds_tab[DS_TAB_ENTRIES];
  {
    const uint4* src = (const uint4*)g_ds_tab.e;
    uint4* dst = (uint4*)ds_tab;
#pragma unroll
    for (int k = 0; k < DS_TAB_ENTRIES / 2 / LAT_BLOCK; ++k)
      dst[k * LAT_BLOCK + threadIdx.x] = src[k * LAT_BLOCK + threadIdx.x];
  }
#endif
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
  // ---- comb waves: LAT_SW signatures per wave, SPLIT lanes each
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
      mrow = msg_idx[(size_t)mi_stride * ii];
      kok = kok && mrow < n_msg;
      if (mrow >= n_msg) mrow = 0;
    }
    s_ok = sc_lt_L(s);
    sc_clamp_rejected(s, s_ok);  // s >= L: recode 0, never index past the base-point table
    uint32_t h[16], k[8];
    sha512_k<LEN>(h, rr, a, msg + (size_t)msg_stride * mrow, (int)msg_len, wk, mrow);
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
  // sum the SPLIT partial points: lanes r ^ 1, r ^ 2 (, r ^ 4) (extended addition, complete formulas)
  auto combine = [&](int m) {
    ge Q, Sum;
    fe_shfl_xor(Q.X, P.X, m); fe_shfl_xor(Q.Y, P.Y, m); fe_shfl_xor(Q.Z, P.Z, m); fe_shfl_xor(Q.T, P.T, m);
    ge_add(Sum, P, Q);
    P = Sum;
  };
  combine(1);
  combine(2);
  if constexpr (SPLIT == 8) combine(4);
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
    // compress R' and compare with the canonical R encoding (DESIGN.md "R check")
    fe zi, x, y;
#if PBFT_LAT_TREE
    // One inversion per wave instead of one per lane: butterfly product of the wave's LAT_SW Z's over
    // lanes ^SPLIT .. ^32 (the SPLIT lanes of a signature hold the same R'), so every lane holds the
    // same product and the shorter variable-time divsteps (inv25519.h) never diverge; the down-sweep
    // peels the partners off again (1 / t_k = (1 / t_{k+1}) q_k).  Z is never 0 (complete formulas
    // over curve points; invalid keys have identity tables), so no lane poisons the others.
    // PBFT_LAT_ROWS: the tree stops at the 16-lane row and each row inverts its own product
    // (fe_invert_wave<true>): two butterfly levels fewer each way, same inversion count per wave
    constexpr int LV = PBFT_LAT_ROWS ? (SPLIT == 4 ? 2 : 1) : (SPLIT == 4 ? 4 : 3);  // log2(signatures per tree)
    fe t = P.Z, tq[LV];
    static_for<LV>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      fe_shfl_xor(tq[k], t, SPLIT << k);
      fe_mul(t, t, tq[k]);
    });
#if PBFT_ABL_NOINV  // ablation: no inversion (timing only, results wrong)
    zi = t;
#elif PBFT_LAT_TAB
    __syncthreads();  // the block's divstep table is in LDS (copied at kernel start)
    #if PBFT_INV_WAVE
    fe_invert_wave<PBFT_LAT_ROWS>(zi, t, ds_tab);  // limbs across lanes, DPP carries (inv25519.h)
#else
    static_assert(!PBFT_LAT_ROWS, "");
    fe_invert_tab(zi, t, ds_tab);
#endif
#else
    fe_invert_var(zi, t);
#endif
    static_for<LV>([&](auto kc) {
      constexpr int k = LV - 1 - decltype(kc)::value;
      fe_mul(zi, zi, tq[k]);
    });
#else
    fe_invert_gcd(zi, P.Z);  // one constant-time divsteps inversion per lane
#endif
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
  // lanes SPLIT j (j < LAT_SW) hold this wave's LAT_SW results: one LAT_SW-bit piece of the bitmap
  // (u16 pieces at 4 lanes per signature, bytes at 8)
  const uint64_t vote = __ballot(acc);
  uint32_t bits = 0;
#pragma unroll
  for (int j = 0; j < LAT_SW; ++j) bits |= (uint32_t)((vote >> (SPLIT * j)) & 1u) << j;
  const uint64_t piece = (uint64_t)blockIdx.x * LAT_COMB_WAVES + wave;  // signatures LAT_SW piece .. + LAT_SW - 1
  if (lane == 0 && piece < (uint64_t)SPLIT * ((N + 63) / 64)) {            // bits past N: 0
    if constexpr (LAT_SW == 16) ((uint16_t*)bitmap)[piece] = (uint16_t)bits;
    else ((uint8_t*)bitmap)[piece] = (uint8_t)bits;
  }
}

// ---- per-plan launchers (comb_paNN.hip) ---------------------------------------
struct comb_launch_args {
  const uint8_t *R, *S, *K;
  uint32_t rs_stride, k_stride;
  const uint8_t* M;
  uint32_t msg_len, msg_stride;
  uint64_t N;
  const uint32_t *tabB, *tabA, *keys;
  const uint8_t* key_ok;
  uint32_t n_keys;
  uint32_t* xyz;           // comb -> finish workspace (one-lane mode)
  uint8_t* flags;
  uint32_t* eidx;          // entry-index workspace (latency mode: 64-bit entry addresses)
  uint64_t* bitmap;        // latency mode writes the bitmap itself
  const uint32_t* msg_idx; // votes form (null: one message per signature)
  uint32_t mi_stride = 1;  // msg_idx[mi_stride * i] (the votes rows layout: PBFT_VOTES_ROW_BYTES / 4)
  uint32_t n_msg;
  const uint64_t* wk;      // votes form, 85-byte envelopes: per-envelope block-2 schedule (null: hash in full)
  bool latency_mode;
  int lat_split;           // latency mode lanes per signature: 4, 8 or 0 (by batch size)
  int pair = -1;           // one-lane mode: comb_pair_kernel 1 / comb_kernel 0 / by batch size -1
  int cus = 0;             // compute units of the device (0: unknown)
  int prio = -1;           // one-lane chain-form comb: 8-wave blocks with paired wave priorities (WPB = 8): 1 on,
                           // 0 off, -1 by batch size
  hipStream_t st;
};

// Even placement of a one-generation launch.  The 131k shard's comb launch is 512 blocks of 4
// waves (128 VGPRs: up to 4 blocks per CU), i.e. 2 per CU if spread evenly -- but the stamped build showed the
// waves ending anywhere between 94 and 148 us after a common start, live waves falling to 0.9 per SIMD over the
// last quarter of the launch (profiles/r05/shard_waits.txt): the dispatcher packs up to 4 blocks onto some CUs
// and leaves others short, and the launch lasts as long as its most crowded SIMD.  Requesting enough LDS that a CU
// holds at most ceil(blocks / CUs) blocks forces the even placement.  Launches of >= 4 blocks per CU keep lds_min.
static inline size_t comb_spread_lds(uint64_t blocks, int cus, size_t lds_min) {
  if (cus <= 0 || blocks == 0) return lds_min;
  const uint64_t per = (blocks + (uint64_t)cus - 1) / (uint64_t)cus;
  // X with per * X <= 160 KB < (per + 1) * X: 1 -> 96 KB, 2 -> 72 KB, 3 -> 48 KB
  const size_t want = per == 1 ? 96 * 1024 : per == 2 ? 72 * 1024 : per == 3 ? 48 * 1024 : 0;
  return want > lds_min ? want : lds_min;
}

// Which one-lane comb a launch runs (launch_comb_plan).
static inline bool comb_pair_sel(const comb_launch_args& a) {
  return a.pair >= 0 ? a.pair > 0 : (a.N >= PBFT_PAIR_MIN_N && a.N <= PBFT_PAIR_MAX_N);
}
// the chain-form comb (85-byte messages, from PBFT_CHAIN_MIN_N signatures)
static inline bool comb_chain(const comb_launch_args& a) {
  return !a.latency_mode && !comb_pair_sel(a) && a.msg_len == PBFT_ENVELOPE_LEN && a.N >= PBFT_CHAIN_MIN_N;
}
// ... in 8-wave blocks with paired priorities: by size, where they fit one per CU (2 waves per SIMD, one
// generation: the 131k shard of an 8-GPU round, -4.3 %); from 2 per CU the SIMDs hold 4 waves and oldest-first
// costs nothing (2^18 -0.7 %, 2^20 +0.3 %), and 1.5 per CU (196,608) would leave half the CUs with twice the
// waves (+14.5 %) (profiles/r05/prio/)
static inline bool comb_chain_prio(const comb_launch_args& a) {
  return comb_chain(a) &&
         (a.prio >= 0 ? a.prio > 0 : (a.cus > 0 && (a.N + 2 * BLOCK - 1) / (2 * BLOCK) <= (uint64_t)a.cus));
}
// Launch the comb (or, in latency mode, the 4-lanes-per-signature kernel) for
// key plan PLA; LEN 85 (the signed envelope) is a specialised template.
template <class PLA>
hipError_t launch_comb_plan(const comb_launch_args& a) {
  const uint64_t N = a.N;
  if (a.latency_mode) {
    const int split = a.lat_split ? a.lat_split : (N <= LAT_WIDE_UPTO ? 8 : 4);
    // enough blocks for every piece of the ceil(N/64) bitmap words (>= ceil(N / signatures per block))
    const uint64_t pieces = (uint64_t)split * ((N + 63) / 64);
    const uint64_t sblocks = (pieces + LAT_COMB_WAVES - 1) / LAT_COMB_WAVES, Lpad = sblocks * LAT_COMB_WAVES * 64;
#define PBFT_LAUNCH_LAT(LEN_, SPL_)                                                                               \
  hipLaunchKernelGGL((comb_latency_kernel<LEN_, PLA, SPL_>), dim3((unsigned)sblocks), dim3(LAT_BLOCK), LAT_LDS, a.st, \
                     a.R, a.S, a.K, a.rs_stride, a.k_stride, a.M, a.msg_len, a.msg_stride, N, Lpad, a.tabB, a.tabA,   \
                     a.keys, a.key_ok, a.n_keys, a.bitmap, (const uint8_t**)a.eidx, a.msg_idx, a.n_msg, a.mi_stride, a.wk)
    if (a.msg_len == PBFT_ENVELOPE_LEN) {
      if (split == 8 && !PBFT_LAT_DECOMP) PBFT_LAUNCH_LAT(PBFT_ENVELOPE_LEN, 8 - 4 * PBFT_LAT_DECOMP);
      else PBFT_LAUNCH_LAT(PBFT_ENVELOPE_LEN, 4);
    } else {
      if (split == 8 && !PBFT_LAT_DECOMP) PBFT_LAUNCH_LAT(-1, 8 - 4 * PBFT_LAT_DECOMP);
      else PBFT_LAUNCH_LAT(-1, 4);
    }
#undef PBFT_LAUNCH_LAT
  } else {
    const uint64_t blocks = (N + BLOCK - 1) / BLOCK, Npad = blocks * BLOCK;
    const bool pair = comb_pair_sel(a);
    const size_t lds = comb_spread_lds(blocks, a.cus, (BLOCK / 64) * COMB_LDS_PER_WAVE);
    if (pair) {
      const uint64_t pblocks = (N + PAIR_SIGS - 1) / PAIR_SIGS;
      const size_t plds = comb_spread_lds(pblocks, a.cus, PAIR_LDS);
#define PBFT_LAUNCH_PAIR(LEN_)                                                                                     \
  hipLaunchKernelGGL((comb_pair_kernel<LEN_, PLA>), dim3((unsigned)pblocks), dim3(BLOCK), plds, a.st, a.R, a.S,     \
                     a.K, a.rs_stride, a.k_stride, a.M, a.msg_len, a.msg_stride, N, Npad, a.tabB, a.tabA, a.keys,    \
                     a.key_ok, a.n_keys, a.xyz, a.flags, a.eidx, a.msg_idx, a.n_msg, a.mi_stride, a.wk)
      if (a.msg_len == PBFT_ENVELOPE_LEN) PBFT_LAUNCH_PAIR(PBFT_ENVELOPE_LEN);
      else PBFT_LAUNCH_PAIR(-1);
#undef PBFT_LAUNCH_PAIR
    } else if (comb_chain_prio(a)) {
      const uint64_t b2 = (N + 2 * BLOCK - 1) / (2 * BLOCK), Npad2 = b2 * 2 * BLOCK;  // (eidx sized for this pad)
      const size_t lds2 = 8 * COMB_LDS_PER_WAVE + COMB_PRIO_LDS;
      hipLaunchKernelGGL((comb_kernel<PBFT_ENVELOPE_LEN, PLA, true, 8>), dim3((unsigned)b2), dim3(2 * BLOCK), lds2,
                         a.st, a.R, a.S, a.K, a.rs_stride, a.k_stride, a.M, a.msg_len, a.msg_stride, N, Npad2, a.tabB,
                         a.tabA, a.keys, a.key_ok, a.n_keys, a.xyz, a.flags, a.eidx, a.msg_idx, a.n_msg, a.mi_stride,
                         a.wk);
    } else if (comb_chain(a)) {
      hipLaunchKernelGGL((comb_kernel<PBFT_ENVELOPE_LEN, PLA, true, 4>), dim3((unsigned)blocks), dim3(BLOCK), lds,
                         a.st, a.R, a.S, a.K, a.rs_stride, a.k_stride, a.M, a.msg_len, a.msg_stride, N, Npad, a.tabB,
                         a.tabA, a.keys, a.key_ok, a.n_keys, a.xyz, a.flags, a.eidx, a.msg_idx, a.n_msg, a.mi_stride,
                         a.wk);
    } else if (a.msg_len == PBFT_ENVELOPE_LEN)
      hipLaunchKernelGGL((comb_kernel<PBFT_ENVELOPE_LEN, PLA>), dim3((unsigned)blocks), dim3(BLOCK), lds, a.st, a.R,
                         a.S, a.K, a.rs_stride, a.k_stride, a.M, a.msg_len, a.msg_stride, N, Npad, a.tabB, a.tabA,
                         a.keys, a.key_ok, a.n_keys, a.xyz, a.flags, a.eidx, a.msg_idx, a.n_msg, a.mi_stride, a.wk);
    else
      hipLaunchKernelGGL((comb_kernel<-1, PLA>), dim3((unsigned)blocks), dim3(BLOCK), lds, a.st, a.R, a.S, a.K,
                         a.rs_stride, a.k_stride, a.M, a.msg_len, a.msg_stride, N, Npad, a.tabB, a.tabA, a.keys,
                         a.key_ok, a.n_keys, a.xyz, a.flags, a.eidx, a.msg_idx, a.n_msg, a.mi_stride, a.wk);
  }
  return hipGetLastError();
}

// defined in comb_pa13.hip / comb_pa14.hip / comb_pa16.hip / comb_pa32.hip
hipError_t launch_comb_huge(const comb_launch_args& a);
hipError_t launch_comb_big(const comb_launch_args& a);
hipError_t launch_comb_mid(const comb_launch_args& a);
hipError_t launch_comb_small(const comb_launch_args& a);

// tables.hip: comb tables of the base point (pa = 0, plan PLB) or of -A per key (pa = the key plan's positions).
// d_slot (optional): key k goes to slot d_slot[k] of d_tables / d_key_ok / d_keys_out (partial rebuild);
// d_keys_out (optional): the raw encodings, stored at their slots.  *wrote (optional) is set to 1 once a kernel
// that writes the tables / key_ok / keys_out has been launched: a failure with *wrote == 0 changed nothing (the
// scratch is allocated before the first launch).
hipError_t build_comb_tables(int pa, const uint32_t* d_enc, uint32_t n, int negate, uint32_t* d_tables,
                             uint8_t* d_key_ok, hipStream_t st, const uint32_t* d_slot = nullptr,
                             uint32_t* d_keys_out = nullptr, int* wrote = nullptr);

// finish.hip: batch-inversion finish of the one-lane comb: fm (1, 2, 4, 8, 16) signatures per lane, lv = 0
// (one inversion per lane) or nonzero (cross-lane product tree of PBFT_FIN_LV levels: one inversion per 16-lane
// row, or per wave), w = waves per SIMD it is compiled for (tree: 1, or 2 for fm 2 / 4 / 8)
hipError_t launch_finish(int fm, int lv, int w, const uint8_t* R, uint32_t rs_stride, const uint32_t* xyz,
                         const uint8_t* flags, uint64_t N, uint64_t* bitmap, hipStream_t st);
// sign.hip: RFC 8032 signing, len = 85 (envelope), 0 (public keys only) or -1 (any length)
void launch_sign(int len, dim3 grid, dim3 block, size_t lds, hipStream_t st, const uint32_t* seeds,
                 const uint16_t* seed_idx, const uint8_t* msg, uint32_t msg_len, uint32_t msg_stride, uint64_t N,
                 const uint32_t* tabB, uint32_t* R, uint32_t* S, uint32_t* pub, uint32_t n_seeds);
