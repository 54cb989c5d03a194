// Batch-inversion finish of the one-lane-per-signature verify (comb_kernel ->
// finish_kernel), its own translation unit.
#include "verify_kernels.h"

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

static_assert(PBFT_FIN_LV == 4 || PBFT_FIN_LV == 6, "");
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

// W: waves per SIMD the kernel is compiled for (register budget 512 / W); the prefetch of X, Y, Z needs W = 1
template <int FM, int LV, int W>
__global__ void __launch_bounds__(BLOCK, W) finish_kernel(const uint8_t* __restrict__ R,
                                                       uint32_t rs_stride,
                                                       const uint32_t* __restrict__ xyz,
                                                       const uint8_t* __restrict__ flags, uint64_t N,
                                                       uint64_t* __restrict__ bitmap) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;
  const uint64_t base = wave * FM * 64 + lane;
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
#endif
  if (wave * FM * 64 >= N) return;
  FIN_STAMP(0);
#if PBFT_FIN_STAMPS
  if (lane == 0 && wave < FIN_STAMP_WAVES) g_fin_stamp[wave][6] = __builtin_amdgcn_s_memrealtime();
#endif
  const uint32_t* Xb = xyz;
  const uint32_t* Yb = xyz + 10 * N;
  const uint32_t* Zb = xyz + 20 * N;
  // prefix products of Z (lanes past N contribute 1)
  fe pre[FM];
  // PRE: small FM keeps every Z and issues the X, Y loads before the inversion, so the back-substitution
  // does not wait on memory (FM <= 4: ~100 more VGPRs, within the 2-waves-per-SIMD budget)
  constexpr bool PRE = PBFT_FIN_PREFETCH && ((FM <= 4 && W == 1) || FM == 1);
  fe zs[PRE ? FM : 1], xs[PRE ? FM : 1], ys[PRE ? FM : 1];
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
    }
    if constexpr (m == 0) pre[0] = z;
    else fe_mul(pre[m], pre[m - 1], z);
  });
  FIN_STAMP(1);
  fe inv;
  fe tq[LV > 0 ? LV : 1];  // partner products of the butterfly levels
  fe t = pre[FM - 1];
  static_for<LV>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
#pragma unroll
    for (int u = 0; u < 10; ++u) tq[k].v[u] = tree_partner<k>(t.v[u]);
    fe_mul(t, t, tq[k]);
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
    __syncthreads();  // the block's divstep table is in LDS
#if PBFT_INV_WAVE
    fe_invert_wave<(LV < 6)>(inv, t, ds_tab);  // limbs across lanes, DPP carries (inv25519.h)
#else
    static_assert(LV == 6, "");
    fe_invert_tab(inv, t, ds_tab);
#endif
#elif PBFT_FIN_STAMPS
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
    fe_mul(inv, inv, tq[k]);  // 1 / (product of this lane's 2^k group)
  });
  FIN_STAMP(4);
  fin_unroll<FM>::down([&](auto mc) {
    constexpr int m = decltype(mc)::value;
    const uint64_t i = base + (uint64_t)m * 64;
    const bool live = i < N;
    const uint64_t ii = live ? i : 0;
    fe zi;
    if constexpr (m > 0) {
      fe_mul(zi, inv, pre[m - 1]);   // 1 / Z_m
      fe z;
      if constexpr (PRE) z = zs[m];
      else if (live) load_fe(z, Zb, N, ii); else fe_one(z);
      fe_mul(inv, inv, z);           // 1 / (Z_0 ... Z_{m-1})
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
  FIN_STAMP(5);
#if PBFT_FIN_STAMPS
  if (lane == 0 && wave < FIN_STAMP_WAVES) g_fin_stamp[wave][7] = __builtin_amdgcn_s_memrealtime();
#endif
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
