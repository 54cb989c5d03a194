// GF(2^255 - 19) arithmetic for gfx950, one field element per lane.
//
// Representation: 10 unsigned limbs in radix 2^25.5 (26,25,26,25,... bits), held
// in 32-bit VGPRs.  Products are 32x32->64 and accumulate with v_mad_u64_u32
// (measured on MI355X: ~1.3x the issue cost of a 32-bit VOP3 op),
// so a multiply is 100 mads + one 64-bit carry chain; a square is 55 mads.
//
// Bounds discipline (checked by tools/limb_bounds.py):
//  * "carried"  : output of fe_mul/fe_sq/fe_carry: limbs <= 2^26 / 2^25 (+2^14 slack)
//  * fe_add     : no carry; inputs carried -> limbs <= 2^27
//  * fe_sub     : f + 2p - g; g must be carried; result limbs <= 3*2^26
//  * fe_mul/sq  : accept any operands produced by one add/sub of carried values;
//                 every 64-bit column stays < 2^63.3.
// Semantics mirrored: curve25519-dalek 3.2.1 FieldElement (Cargo.lock:604-614).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef FE_FN
#define FE_FN __host__ __device__ __forceinline__
#endif

namespace pbft {

struct fe { uint32_t v[10]; };

#define M26 0x3FFFFFFu
#define M25 0x1FFFFFFu

FE_FN void fe_zero(fe& h) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = 0;
}
FE_FN void fe_one(fe& h) { fe_zero(h); h.v[0] = 1; }

FE_FN void fe_add(fe& h, const fe& f, const fe& g) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] + g.v[i];
}

// h = f - g + 2p  (g carried)
FE_FN void fe_sub(fe& h, const fe& f, const fe& g) {
  h.v[0] = f.v[0] + 0x7FFFFDAu - g.v[0];
#pragma unroll
  for (int i = 1; i < 10; ++i) h.v[i] = f.v[i] + ((i & 1) ? 0x3FFFFFEu : 0x7FFFFFEu) - g.v[i];
}

// h = -f  (f carried)
FE_FN void fe_neg(fe& h, const fe& f) {
  h.v[0] = 0x7FFFFDAu - f.v[0];
#pragma unroll
  for (int i = 1; i < 10; ++i) h.v[i] = ((i & 1) ? 0x3FFFFFEu : 0x7FFFFFEu) - f.v[i];
}

// one carry pass over u32 limbs (inputs < 2^31)
FE_FN void fe_carry(fe& h) {
  uint32_t c;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int sh = (i & 1) ? 25 : 26;
    c = h.v[i] >> sh; h.v[i] &= (i & 1) ? M25 : M26; h.v[i + 1] += c;
  }
  c = h.v[9] >> 25; h.v[9] &= M25; h.v[0] += 19u * c;
  c = h.v[0] >> 26; h.v[0] &= M26; h.v[1] += c;
}

#define MUL64(a, b) ((uint64_t)(a) * (uint64_t)(b))
#ifndef PBFT_REDUCE_1CHAIN
#define PBFT_REDUCE_1CHAIN 1  // A/B r03: -2.0 % on the 131k shard, -0.7 % at 2^20 (profiles/r03/ab_chain1.txt)
#endif

FE_FN void fe_reduce_wide(fe& h, uint64_t h0, uint64_t h1, uint64_t h2, uint64_t h3,
                                               uint64_t h4, uint64_t h5, uint64_t h6, uint64_t h7,
                                               uint64_t h8, uint64_t h9) {
  uint64_t c;
#if PBFT_REDUCE_1CHAIN
  // one chain 0 -> 1 -> ... -> 9 -> 0 (x19) -> 1: 11 carries instead of 12, dependency depth 11 instead of 7
  c = h0 >> 26; h1 += c; h0 &= M26;
  c = h1 >> 25; h2 += c; h1 &= M25;
  c = h2 >> 26; h3 += c; h2 &= M26;
  c = h3 >> 25; h4 += c; h3 &= M25;
  c = h4 >> 26; h5 += c; h4 &= M26;
  c = h5 >> 25; h6 += c; h5 &= M25;
  c = h6 >> 26; h7 += c; h6 &= M26;
  c = h7 >> 25; h8 += c; h7 &= M25;
  c = h8 >> 26; h9 += c; h8 &= M26;
  c = h9 >> 25; h0 += c * 19u; h9 &= M25;
  c = h0 >> 26; h1 += c; h0 &= M26;
  h.v[0] = (uint32_t)h0; h.v[1] = (uint32_t)h1; h.v[2] = (uint32_t)h2; h.v[3] = (uint32_t)h3;
  h.v[4] = (uint32_t)h4; h.v[5] = (uint32_t)h5; h.v[6] = (uint32_t)h6; h.v[7] = (uint32_t)h7;
  h.v[8] = (uint32_t)h8; h.v[9] = (uint32_t)h9;
  return;
#endif
  c = h0 >> 26; h1 += c; h0 &= M26;
  c = h4 >> 26; h5 += c; h4 &= M26;
  c = h1 >> 25; h2 += c; h1 &= M25;
  c = h5 >> 25; h6 += c; h5 &= M25;
  c = h2 >> 26; h3 += c; h2 &= M26;
  c = h6 >> 26; h7 += c; h6 &= M26;
  c = h3 >> 25; h4 += c; h3 &= M25;
  c = h7 >> 25; h8 += c; h7 &= M25;
  c = h4 >> 26; h5 += c; h4 &= M26;
  c = h8 >> 26; h9 += c; h8 &= M26;
  c = h9 >> 25; h0 += c * 19u; h9 &= M25;
  c = h0 >> 26; h1 += c; h0 &= M26;
  h.v[0] = (uint32_t)h0; h.v[1] = (uint32_t)h1; h.v[2] = (uint32_t)h2; h.v[3] = (uint32_t)h3;
  h.v[4] = (uint32_t)h4; h.v[5] = (uint32_t)h5; h.v[6] = (uint32_t)h6; h.v[7] = (uint32_t)h7;
  h.v[8] = (uint32_t)h8; h.v[9] = (uint32_t)h9;
}

// Latency-oriented reduction of the 10 64-bit columns: every carry of a round is
// computed at once (two rounds), so the dependent chain is ~4 operations deep
// instead of the 12 sequential carries of fe_reduce_wide (~40 % more
// instructions).  For code that runs one wave per SIMD on a serial chain -- the
// inversion of the finish kernel, R decompression in the latency kernel -- where
// VALU latency, not issue, is the bound.  Output limbs <= 2^26 + 2^17.6
// (limb 0) / 2^25 + 2^16.6 (limb 1) / 2^26 + 2^13.4: within every bound fe_sub
// and fe_mul need (tools/limb_bounds.py, host harness tests).
FE_FN void fe_reduce_par(fe& h, uint64_t c[10]) {
  uint64_t q[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    q[k] = c[k] >> ((k & 1) ? 25 : 26);
    c[k] &= (k & 1) ? M25 : M26;
  }
  c[0] += q[9] * 19u;
#pragma unroll
  for (int k = 1; k < 10; ++k) c[k] += q[k - 1];
  uint32_t r[10], l[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    r[k] = (uint32_t)(c[k] >> ((k & 1) ? 25 : 26));
    l[k] = (uint32_t)c[k] & ((k & 1) ? M25 : M26);
  }
  h.v[0] = l[0] + 19u * r[9];
#pragma unroll
  for (int k = 1; k < 10; ++k) h.v[k] = l[k] + r[k - 1];
}

// 2x as an addition: v_add_u32_e32 issues at ~2.2 cycles per wave64 on gfx950,
// the v_lshlrev_b32 LLVM canonicalises x + x into at ~4.0
// (tools/microbench/valu_mix2.hip, profiles/r02_valu_mix2.txt).
FE_FN uint32_t dbl32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_add_u32_e32 %0, %1, %1" : "=v"(r) : "v"(x));
  return r;
#else
  return 2u * x;
#endif
}

// Operand-scanning order: the 10 column accumulators are updated round-robin,
// so consecutive v_mad_u64_u32 never depend on each other (10-way ILP per lane;
// the dependent-mad latency is ~17 cycles on gfx950, tools/microbench/mad_latency.hip).
FE_FN void fe_mul_cols(uint64_t acc[10], const fe& f, const fe& g) {
  uint32_t g19[10], fx[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    g19[i] = 19u * g.v[i];
    fx[i] = (i & 1) ? dbl32(f.v[i]) : f.v[i];
  }
#pragma unroll
  for (int k = 0; k < 10; ++k) acc[k] = MUL64(f.v[0], g.v[k]);
#pragma unroll
  for (int i = 1; i < 10; ++i) {
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      const int j = k - i;  // g index; j < 0 wraps with x19
      // odd*odd limb products carry an extra factor 2 (radix 2^25.5)
      const uint32_t fi = ((i & 1) && (j & 1)) ? fx[i] : f.v[i];
      const uint32_t gj = j >= 0 ? g.v[j] : g19[j + 10];
#if defined(__HIP_DEVICE_COMPILE__) && defined(PBFT_ASM_MAD)
      // issue order pinned: the machine scheduler otherwise regroups the mads
      // into 4-5 dependent chains
      uint64_t cc;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(cc) : "v"(fi), "v"(gj));
#else
      acc[k] += MUL64(fi, gj);
#endif
    }
  }
}
FE_FN void fe_mul(fe& h, const fe& f, const fe& g) {
  uint64_t acc[10];
  fe_mul_cols(acc, f, g);
  fe_reduce_wide(h, acc[0], acc[1], acc[2], acc[3], acc[4], acc[5], acc[6], acc[7], acc[8], acc[9]);
}

// acc' = a * b + acc with the accumulator pinned as the mad's addend, so that LLVM cannot re-associate a carry
// that starts the chain into a separate 64-bit add.
// acc' = a * b + acc, laundered: the opaque result keeps LLVM from re-associating a chain that starts with a
// carry (it would add the carry last, as a separate 64-bit add); the add still folds into the v_mad_u64_u32.
// (Writing the mad itself as inline asm was slower: its SGPR carry-out makes the hazard recognizer pad every
// asm boundary with an s_nop.)
FE_FN uint64_t mad_acc(uint32_t a, uint32_t b, uint64_t acc) {
  acc += MUL64(a, b);
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(acc));
#endif
  return acc;
}

#ifndef PBFT_CHAIN_FORM
#define PBFT_CHAIN_FORM 0
#endif
#ifndef PBFT_COLUMN_ASM
#define PBFT_COLUMN_ASM 1  // fe_mul_chain: one inline-asm block of 10 mads per (product, column)
#endif

// One column of a single-chain product (fe_mul_chain), device code: acc' = acc + sum_i fi[i] * gj[i] as TEN
// v_mad_u64_u32 in ONE inline-asm block (FIRST: acc' = sum, no addend).  The block is opaque to LLVM, so the carry
// that enters as the first mad's addend is never re-associated into a separate 64-bit add -- what the per-mad
// laundering asm of mad_acc() achieved at the price of one hazard s_nop after nearly every mad: gfx950's
// DstSel-forwarding hazard check assumes an inline-asm def may need one wait state before the next VALU that
// touches it, so 715 launders per comb step cost 247 s_nop (profiles/r03/step_hist_chain.txt); one asm per
// column leaves at most one per column, usually none (the other products' columns fill the slot).
#if defined(__HIP_DEVICE_COMPILE__)
template <bool FIRST>
__device__ __forceinline__ void mad_column10(uint64_t& acc, const uint32_t fi[10], const uint32_t gj[10]) {
  uint64_t cc;
#define PBFT_MAD_COL_REST                                                                                         \
  "v_mad_u64_u32 %0, %1, %4, %5, %0\n\t"                                                                            \
  "v_mad_u64_u32 %0, %1, %6, %7, %0\n\t"                                                                            \
  "v_mad_u64_u32 %0, %1, %8, %9, %0\n\t"                                                                            \
  "v_mad_u64_u32 %0, %1, %10, %11, %0\n\t"                                                                          \
  "v_mad_u64_u32 %0, %1, %12, %13, %0\n\t"                                                                          \
  "v_mad_u64_u32 %0, %1, %14, %15, %0\n\t"                                                                          \
  "v_mad_u64_u32 %0, %1, %16, %17, %0\n\t"                                                                          \
  "v_mad_u64_u32 %0, %1, %18, %19, %0\n\t"                                                                          \
  "v_mad_u64_u32 %0, %1, %20, %21, %0"
#define PBFT_MAD_COL_IN                                                                                           \
  "v"(fi[0]), "v"(gj[0]), "v"(fi[1]), "v"(gj[1]), "v"(fi[2]), "v"(gj[2]), "v"(fi[3]), "v"(gj[3]), "v"(fi[4]),    \
      "v"(gj[4]), "v"(fi[5]), "v"(gj[5]), "v"(fi[6]), "v"(gj[6]), "v"(fi[7]), "v"(gj[7]), "v"(fi[8]), "v"(gj[8]), \
      "v"(fi[9]), "v"(gj[9])
  if constexpr (FIRST)
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0\n\t" PBFT_MAD_COL_REST : "=&v"(acc), "=&s"(cc) : PBFT_MAD_COL_IN);
  else
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n\t" PBFT_MAD_COL_REST : "+v"(acc), "=&s"(cc) : PBFT_MAD_COL_IN);
#undef PBFT_MAD_COL_REST
#undef PBFT_MAD_COL_IN
  (void)cc;
}
#endif
// N independent products h[m] = f[m] g[m], each computed as ONE dependent chain over the columns: column k's
// mads accumulate on top of column k-1's carry, so a carry costs one 64-bit shift and one mask and no 64-bit
// add (fe_reduce_wide's single-chain arithmetic, PBFT_REDUCE_1CHAIN: identical outputs and bounds).  The N
// chains are interleaved product by product, so a wave has N independent mads in flight.  For the comb step
// of large batches (comb_kernel<..., CHAIN>); latency-bound code (one wave per SIMD) keeps fe_mul.
template <int N>
FE_FN void fe_mul_chain(fe* const h[], const fe* const f[], const fe* const g[]) {
  uint32_t g19[N][10], fx[N][10], l[N][10];
  uint64_t acc[N];
#pragma unroll
  for (int m = 0; m < N; ++m) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      g19[m][i] = 19u * g[m]->v[i];
      fx[m][i] = (i & 1) ? dbl32(f[m]->v[i]) : f[m]->v[i];
    }
  }
#if defined(__HIP_DEVICE_COMPILE__) && PBFT_COLUMN_ASM
#ifndef PBFT_COLUMN_ASM_MOUTER
#define PBFT_COLUMN_ASM_MOUTER 1
#endif
#pragma unroll
  for (int kk = 0; kk < 10 * N; ++kk) {
    // product by product (m outer): one product's operands live at a time; else column by column
    const int k = PBFT_COLUMN_ASM_MOUTER ? kk % 10 : kk / N;
    const int m = PBFT_COLUMN_ASM_MOUTER ? kk / 10 : kk % N;
    {
      uint32_t fi[10], gj[10];
#pragma unroll
      for (int i = 0; i < 10; ++i) {
        const int j = k - i;  // g index; j < 0 wraps with x19; odd*odd limb products carry an extra factor 2
        fi[i] = ((i & 1) && (j & 1)) ? fx[m][i] : f[m]->v[i];
        gj[i] = j >= 0 ? g[m]->v[j] : g19[m][j + 10];
      }
      if (k == 0) mad_column10<true>(acc[m], fi, gj);
      else mad_column10<false>(acc[m], fi, gj);
      l[m][k] = (uint32_t)acc[m] & ((k & 1) ? M25 : M26);
      acc[m] >>= (k & 1) ? 25 : 26;
    }
  }
#else
#pragma unroll
  for (int k = 0; k < 10; ++k) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const int j = k - i;  // g index; j < 0 wraps with x19
      uint32_t fi[N], gj[N];
#pragma unroll
      for (int m = 0; m < N; ++m) {
        fi[m] = ((i & 1) && (j & 1)) ? fx[m][i] : f[m]->v[i];
        gj[m] = j >= 0 ? g[m]->v[j] : g19[m][j + 10];
      }
#if PBFT_CHAIN_FORM == 0
#pragma unroll
      for (int m = 0; m < N; ++m) acc[m] = (k == 0 && i == 0) ? MUL64(fi[m], gj[m]) : mad_acc(fi[m], gj[m], acc[m]);
#else
      // launder only the carry that starts a column (its first mad takes it as the addend); the column's other
      // mads chain on that one
#pragma unroll
      for (int m = 0; m < N; ++m) {
        if (k == 0 && i == 0) acc[m] = MUL64(fi[m], gj[m]);
        else if (i == 0) acc[m] = mad_acc(fi[m], gj[m], acc[m]);
        else acc[m] += MUL64(fi[m], gj[m]);
      }
#if PBFT_CHAIN_FORM == 2 && defined(__HIP_DEVICE_COMPILE__)
      // one mad of each chain in turn: no two dependent mads back to back
#pragma unroll
      for (int m = 0; m < N; ++m) __builtin_amdgcn_sched_group_barrier(0x2, 1, 0);
#endif
#endif
    }
#pragma unroll
    for (int m = 0; m < N; ++m) {
      l[m][k] = (uint32_t)acc[m] & ((k & 1) ? M25 : M26);
      acc[m] >>= (k & 1) ? 25 : 26;
    }
  }
#endif
#pragma unroll
  for (int m = 0; m < N; ++m) {
    const uint64_t h0 = (uint64_t)l[m][0] + acc[m] * 19u;  // acc = the carry out of column 9
    l[m][1] += (uint32_t)(h0 >> 26);
    l[m][0] = (uint32_t)h0 & M26;
#pragma unroll
    for (int i = 0; i < 10; ++i) h[m]->v[i] = l[m][i];
  }
}

FE_FN void fe_sq_cols(uint64_t c[10], const fe& f) {
  const uint32_t f0 = f.v[0], f1 = f.v[1], f2 = f.v[2], f3 = f.v[3], f4 = f.v[4];
  const uint32_t f5 = f.v[5], f6 = f.v[6], f7 = f.v[7], f8 = f.v[8], f9 = f.v[9];
  const uint32_t f0_2 = 2u * f0, f1_2 = 2u * f1, f2_2 = 2u * f2, f3_2 = 2u * f3, f4_2 = 2u * f4;
  const uint32_t f5_2 = 2u * f5, f6_2 = 2u * f6, f7_2 = 2u * f7;
  const uint32_t f5_38 = 38u * f5, f6_19 = 19u * f6, f7_38 = 38u * f7, f8_19 = 19u * f8, f9_38 = 38u * f9;

  uint64_t h0 = MUL64(f0, f0) + MUL64(f1_2, f9_38) + MUL64(f2_2, f8_19) + MUL64(f3_2, f7_38) +
                MUL64(f4_2, f6_19) + MUL64(f5, f5_38);
  uint64_t h1 = MUL64(f0_2, f1) + MUL64(f2, f9_38) + MUL64(f3_2, f8_19) + MUL64(f4, f7_38) + MUL64(f5_2, f6_19);
  uint64_t h2 = MUL64(f0_2, f2) + MUL64(f1_2, f1) + MUL64(f3_2, f9_38) + MUL64(f4_2, f8_19) +
                MUL64(f5_2, f7_38) + MUL64(f6, f6_19);
  uint64_t h3 = MUL64(f0_2, f3) + MUL64(f1_2, f2) + MUL64(f4, f9_38) + MUL64(f5_2, f8_19) + MUL64(f6, f7_38);
  uint64_t h4 = MUL64(f0_2, f4) + MUL64(f1_2, f3_2) + MUL64(f2, f2) + MUL64(f5_2, f9_38) +
                MUL64(f6_2, f8_19) + MUL64(f7, f7_38);
  uint64_t h5 = MUL64(f0_2, f5) + MUL64(f1_2, f4) + MUL64(f2_2, f3) + MUL64(f6, f9_38) + MUL64(f7_2, f8_19);
  uint64_t h6 = MUL64(f0_2, f6) + MUL64(f1_2, f5_2) + MUL64(f2_2, f4) + MUL64(f3_2, f3) +
                MUL64(f7_2, f9_38) + MUL64(f8, f8_19);
  uint64_t h7 = MUL64(f0_2, f7) + MUL64(f1_2, f6) + MUL64(f2_2, f5) + MUL64(f3_2, f4) + MUL64(f8, f9_38);
  uint64_t h8 = MUL64(f0_2, f8) + MUL64(f1_2, f7_2) + MUL64(f2_2, f6) + MUL64(f3_2, f5_2) +
                MUL64(f4, f4) + MUL64(f9, f9_38);
  uint64_t h9 = MUL64(f0_2, f9) + MUL64(f1_2, f8) + MUL64(f2_2, f7) + MUL64(f3_2, f6) + MUL64(f4_2, f5);
  c[0] = h0; c[1] = h1; c[2] = h2; c[3] = h3; c[4] = h4; c[5] = h5; c[6] = h6; c[7] = h7; c[8] = h8; c[9] = h9;
}
FE_FN void fe_sq(fe& h, const fe& f) {
  uint64_t c[10];
  fe_sq_cols(c, f);
  fe_reduce_wide(h, c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], c[8], c[9]);
}
// PAR = latency-oriented reduction (fe_reduce_par)
template <bool PAR>
FE_FN void fe_sqT(fe& h, const fe& f) {
  if constexpr (PAR) { uint64_t c[10]; fe_sq_cols(c, f); fe_reduce_par(h, c); }
  else fe_sq(h, f);
}
template <bool PAR>
FE_FN void fe_mulT(fe& h, const fe& f, const fe& g) {
  if constexpr (PAR) { uint64_t c[10]; fe_mul_cols(c, f, g); fe_reduce_par(h, c); }
  else fe_mul(h, f, g);
}

template <bool PAR = false>
FE_FN void fe_sqn(fe& h, const fe& f, int n) {
  fe_sqT<PAR>(h, f);
  for (int i = 1; i < n; ++i) fe_sqT<PAR>(h, h);
}

// z^(2^250 - 1) and z^11 (shared by invert and pow22523)
template <bool PAR = false>
FE_FN void fe_pow250(fe& out, fe& z11, const fe& z) {
  fe t0, t1, z9, z2_5_0, z2_10_0, z2_20_0, z2_50_0;
  fe_sqT<PAR>(t1, z);                       // z^2
  fe_sqT<PAR>(t0, t1); fe_sqT<PAR>(t0, t0); // z^8
  fe_mulT<PAR>(z9, t0, z);                  // z^9
  fe_mulT<PAR>(z11, z9, t1);                // z^11
  fe_sqT<PAR>(t0, z11);                     // z^22
  fe_mulT<PAR>(z2_5_0, t0, z9);             // z^31 = z^(2^5-1)
  fe_sqn<PAR>(t0, z2_5_0, 5); fe_mulT<PAR>(z2_10_0, t0, z2_5_0);
  fe_sqn<PAR>(t0, z2_10_0, 10); fe_mulT<PAR>(z2_20_0, t0, z2_10_0);
  fe_sqn<PAR>(t0, z2_20_0, 20); fe_mulT<PAR>(t1, t0, z2_20_0);
  fe_sqn<PAR>(t0, t1, 10); fe_mulT<PAR>(z2_50_0, t0, z2_10_0);
  fe_sqn<PAR>(t0, z2_50_0, 50); fe_mulT<PAR>(t1, t0, z2_50_0);   // 2^100 - 1
  fe_sqn<PAR>(t0, t1, 100); fe_mulT<PAR>(t1, t0, t1);            // 2^200 - 1
  fe_sqn<PAR>(t0, t1, 50); fe_mulT<PAR>(out, t0, z2_50_0);       // 2^250 - 1
}

template <bool PAR = false>
FE_FN void fe_invert(fe& out, const fe& z) {
  fe t, z11;
  fe_pow250<PAR>(t, z11, z);
  fe_sqn<PAR>(t, t, 5);
  fe_mulT<PAR>(out, t, z11);  // z^(2^255 - 21) = z^(p-2)
}

template <bool PAR = false>
FE_FN void fe_pow22523(fe& out, const fe& z) {
  fe t, z11;
  fe_pow250<PAR>(t, z11, z);
  fe_sqn<PAR>(t, t, 2);
  fe_mulT<PAR>(out, t, z);    // z^(2^252 - 3) = z^((p-5)/8)
}

// Fully reduce to the canonical representative < p, as 8 little-endian u32 words.
FE_FN void fe_to_words(uint32_t w[8], const fe& f) {
  fe t = f;
  fe_carry(t);
  fe_carry(t);
  // q = 1 iff t >= p
  uint32_t q = (t.v[0] + 19u) >> 26;
#pragma unroll
  for (int i = 1; i < 10; ++i) q = (t.v[i] + q) >> ((i & 1) ? 25 : 26);
  t.v[0] += 19u * q;
  uint32_t c;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int sh = (i & 1) ? 25 : 26;
    c = t.v[i] >> sh; t.v[i] &= (i & 1) ? M25 : M26; t.v[i + 1] += c;
  }
  t.v[9] &= M25;
  // pack: limb i starts at bit offsets 0,26,51,77,102,128,153,179,204,230
  w[0] = t.v[0] | (t.v[1] << 26);
  w[1] = (t.v[1] >> 6) | (t.v[2] << 19);
  w[2] = (t.v[2] >> 13) | (t.v[3] << 13);
  w[3] = (t.v[3] >> 19) | (t.v[4] << 6);
  w[4] = t.v[5] | (t.v[6] << 25);
  w[5] = (t.v[6] >> 7) | (t.v[7] << 19);
  w[6] = (t.v[7] >> 13) | (t.v[8] << 12);
  w[7] = (t.v[8] >> 20) | (t.v[9] << 6);
}

// Load 8 LE u32 words (bit 255 ignored, value NOT reduced: dalek from_bytes)
FE_FN void fe_from_words(fe& h, const uint32_t w[8]) {
  h.v[0] = w[0] & M26;
  h.v[1] = ((w[0] >> 26) | (w[1] << 6)) & M25;
  h.v[2] = ((w[1] >> 19) | (w[2] << 13)) & M26;
  h.v[3] = ((w[2] >> 13) | (w[3] << 19)) & M25;
  h.v[4] = (w[3] >> 6) & M26;
  h.v[5] = w[4] & M25;
  h.v[6] = ((w[4] >> 25) | (w[5] << 7)) & M26;
  h.v[7] = ((w[5] >> 19) | (w[6] << 13)) & M25;
  h.v[8] = ((w[6] >> 12) | (w[7] << 20)) & M26;
  h.v[9] = (w[7] >> 6) & M25;
}

FE_FN bool fe_is_zero(const fe& f) {
  uint32_t w[8];
  fe_to_words(w, f);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= w[i];
  return o == 0;
}

FE_FN bool fe_is_negative(const fe& f) {
  uint32_t w[8];
  fe_to_words(w, f);
  return w[0] & 1;
}

FE_FN bool fe_eq(const fe& a, const fe& b) {
  fe d;
  fe t = b;
  fe_carry(t);
  fe_sub(d, a, t);
  return fe_is_zero(d);
}

FE_FN void fe_cmov(fe& h, const fe& f, bool c) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = c ? f.v[i] : h.v[i];
}

}  // namespace pbft
