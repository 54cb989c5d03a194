// Batch-inversion finish of the one-lane-per-signature verify, as a per-wave device function run by finish_kernel
// (finish.hip, after comb_kernel).
#pragma once
#include "verify_core.h"

#ifndef FIN_STAMP
#define FIN_STAMP(k)
#endif

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
//
// LV > 0: the lanes' products are also batched ACROSS the wave by a butterfly
// product tree (level k: partner lane l ^ 2^k, one shuffle + one multiply;
// the partner values are kept), so that one inversion serves 2^LV lanes
// instead of one: per signature (FM - 1) + 2 LV / FM + 2 (FM - 1) + 2
// multiplications and 1 / (2^LV FM) of an inversion, instead of 3 (FM - 1) + 2
// and 1 / FM.  The down-sweep peels the partners off again:
// 1 / t_k = (1 / t_{k+1}) q_k, since t_{k+1} = t_k q_k.
#ifndef PBFT_FIN_PREFETCH
#define PBFT_FIN_PREFETCH 1
#endif
#ifndef PBFT_FIN_TAB
#define PBFT_FIN_TAB 1  // LV = 6: table-driven divsteps (inv25519.h fe_invert_tab) instead of divsteps30_var
#endif
#define FIN_USE_TAB (PBFT_FIN_TAB && !PBFT_ABL_NOINV && !PBFT_FIN_EXP)
static_assert(PBFT_FIN_LV == 4 || PBFT_FIN_LV == 6, "");
#ifndef PBFT_FIN_PREFETCH_R
#define PBFT_FIN_PREFETCH_R 0  // 1: (PRE) R and the flag loaded up front too -- r06: no faster at the shard (the wait moves)
#endif
#ifndef PBFT_FIN_PAR
#define PBFT_FIN_PAR 0  // 1: the tree and back-substitution products with the latency-oriented reduction (fe_reduce_par)
#endif
#ifndef PBFT_FIN_DPP
#define PBFT_FIN_DPP 0  // 1: product-tree partners by DPP / ds_swizzle instead of ds_bpermute (r04 A/B: no difference)
#endif
// The partner of this lane at butterfly level k of a product tree over the wave: any involution that pairs the
// level's two 2^k-lane halves of every 2^(k+1)-lane group works (after level k every lane holds the product of
// its group).  Levels 0-3 in-row DPP (quad_perm [1,0,3,2] / [2,3,0,1], row_half_mirror l -> 7-l, row_mirror
// l -> 15-l: a VALU op, no LDS round trip), level 4 ds_swizzle xor 16 (no LDS memory access), level 5
// ds_bpermute xor 32.
template <int K>
__device__ __forceinline__ uint32_t tree_partner(uint32_t v) {
#if PBFT_FIN_DPP
  if constexpr (K == 0) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
  else if constexpr (K == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
  else if constexpr (K == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);
  else if constexpr (K == 3) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);
  else if constexpr (K == 4) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (0x10 << 10) | 0x1F);
  else
#endif
    return (uint32_t)__shfl_xor((int)v, 1 << K);
}


// One wave of the finish: signatures i = (wave * FM + m) * 64 + lane, m < FM; writes their bitmap words.
// PRE: X, Y, Z loaded up front (register budget permitting).  SYNC: meet the block's barrier (the divstep table's
// copy to LDS) right before the inversion -- every wave of the block, past N included, must then reach one
// __syncthreads() (finish_kernel); without SYNC the table is in LDS already.
template <int FM, int LV, bool PRE, bool SYNC>
__device__ __forceinline__ void finish_wave(uint64_t wave, int lane, const uint8_t* __restrict__ R, uint32_t rs_stride,
                                            const uint32_t* __restrict__ xyz, const uint8_t* __restrict__ flags,
                                            uint64_t N, uint64_t* __restrict__ bitmap, const uint64_t* ds_tab) {
  (void)ds_tab; (void)flags;
  const uint64_t base = wave * FM * 64 + lane;
  FIN_STAMP(0);
#if PBFT_FIN_STAMPS && defined(FIN_STAMP_WAVES)
  if (lane == 0 && wave < FIN_STAMP_WAVES) g_fin_stamp[wave][6] = __builtin_amdgcn_s_memrealtime();
#endif
  const uint32_t* Xb = xyz;
  const uint32_t* Yb = xyz + 10 * N;
  const uint32_t* Zb = xyz + 20 * N;
  // prefix products of Z (lanes past N contribute 1)
  fe pre[FM];
  fe zs[PRE ? FM : 1], xs[PRE ? FM : 1], ys[PRE ? FM : 1];
  constexpr bool PRE_R = PRE && PBFT_FIN_PREFETCH_R;
  uint32_t rs[PRE_R ? FM : 1][8];
  bool fls[PRE_R ? FM : 1];
  fin_unroll<FM>::up([&](auto mc) {
    constexpr int m = decltype(mc)::value;
    const uint64_t i = base + (uint64_t)m * 64;
    fe z;
    if (i < N) load_fe(z, Zb, N, i); else fe_one(z);
    if constexpr (PRE) {
      zs[m] = z;
      const uint64_t ii = i < N ? i : 0;
      load_fe(xs[m], Xb, N, ii);
      load_fe(ys[m], Yb, N, ii);
      if constexpr (PRE_R) {  // (issued before the inversion: the compare no longer waits on memory at the end)
        load32(rs[m], R + (size_t)rs_stride * ii);
        fls[m] = flags[ii];
      }
    }
    if constexpr (m == 0) pre[0] = z;
    else fe_mulT<PBFT_FIN_PAR>(pre[m], pre[m - 1], z);
  });
  FIN_STAMP(1);
  fe inv;
  fe tq[LV > 0 ? LV : 1];  // partner products of the butterfly levels
  fe t = pre[FM - 1];
  static_for<LV>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
#pragma unroll
    for (int u = 0; u < 10; ++u) tq[k].v[u] = tree_partner<k>(t.v[u]);
    fe_mulT<PBFT_FIN_PAR>(t, t, tq[k]);
  });
  FIN_STAMP(2);
#if PBFT_ABL_NOINV  // ablation: no inversion (timing only, results wrong)
  inv = t;
#elif PBFT_FIN_EXP  // A/B: z^(p-2) with latency-oriented carries
  fe_invert<true>(inv, t);
#else
  if constexpr (LV > 0) {
    // every lane holds the product of its wave (LV 6) or row (LV 4): the variable-time divsteps never diverge
    // (inv25519.h)
#if FIN_USE_TAB
    if constexpr (SYNC) __syncthreads();  // the block's divstep table is in LDS
#if PBFT_INV_WAVE
    fe_invert_wave<(LV < 6)>(inv, t, ds_tab);  // limbs across lanes, DPP carries (inv25519.h)
#else
    static_assert(LV == 6, "");
    fe_invert_tab(inv, t, ds_tab);
#endif
#elif PBFT_FIN_STAMPS && defined(FIN_STAMP_WAVES)
    static_assert(LV == 6, "");
    uint64_t prof[3];
    fe_invert_var(inv, t, prof);
    if (lane == 0 && wave < FIN_STAMP_WAVES) {
      g_fin_stamp[wave][8] = prof[0]; g_fin_stamp[wave][9] = prof[1]; g_fin_stamp[wave][10] = prof[2];
    }
#else
    static_assert(LV == 6, "");
    fe_invert_var(inv, t);
#endif
  } else {
    fe_invert_gcd(inv, t);  // divsteps: ~19k instructions instead of ~44k on the serial chain
  }
#endif
  FIN_STAMP(3);
  static_for<LV>([&](auto kc) {
    constexpr int k = LV - 1 - decltype(kc)::value;
    fe_mulT<PBFT_FIN_PAR>(inv, inv, tq[k]);  // 1 / (product of this lane's 2^k group)
  });
  FIN_STAMP(4);
  fin_unroll<FM>::down([&](auto mc) {
    constexpr int m = decltype(mc)::value;
    const uint64_t i = base + (uint64_t)m * 64;
    const bool live = i < N;
    const uint64_t ii = live ? i : 0;
    fe zi;
    if constexpr (m > 0) {
      fe_mulT<PBFT_FIN_PAR>(zi, inv, pre[m - 1]);   // 1 / Z_m
      fe z;
      if constexpr (PRE) z = zs[m];
      else if (live) load_fe(z, Zb, N, ii); else fe_one(z);
      fe_mulT<PBFT_FIN_PAR>(inv, inv, z);           // 1 / (Z_0 ... Z_{m-1})
    } else {
      zi = inv;
    }
    fe X, Y, x, y;
    if constexpr (PRE) {
      X = xs[m];
      Y = ys[m];
    } else {
      load_fe(X, Xb, N, ii);
      load_fe(Y, Yb, N, ii);
    }
    bool fl;
    uint32_t r[8];
    if constexpr (PRE_R) {
      fl = fls[m];
#pragma unroll
      for (int t = 0; t < 8; ++t) r[t] = rs[m][t];
    } else {
      fl = flags[ii];
      load32(r, R + (size_t)rs_stride * ii);
    }
    fe_mulT<PBFT_FIN_PAR>(x, X, zi);
    fe_mulT<PBFT_FIN_PAR>(y, Y, zi);
    uint32_t xw[8], yw[8], ry[8];
    fe_to_words(xw, x);
    fe_to_words(yw, y);
    canon_y(ry, r);
    bool eq = (xw[0] & 1u) == (r[7] >> 31);
#pragma unroll
    for (int t = 0; t < 8; ++t) eq = eq && yw[t] == ry[t];
    const bool ok = live && fl && eq && !y_is_small_order(yw);
    const uint64_t vote = __ballot(ok);
    if (lane == 0 && live) bitmap[(wave * FM + m)] = vote;
  });
  FIN_STAMP(5);
#if PBFT_FIN_STAMPS && defined(FIN_STAMP_WAVES)
  if (lane == 0 && wave < FIN_STAMP_WAVES) g_fin_stamp[wave][7] = __builtin_amdgcn_s_memrealtime();
#endif
}
