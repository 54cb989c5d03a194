// Per-lane Ed25519 verify_strict for the PBFT prepare/commit hot path.
//
// Replaces the signature TODOs of the reference's validators
// (src/behavior.rs:127, :185; slots validate_prepare :159-175 and
// validate_commit :184-195) with ed25519-dalek 1.0.1 verify_strict semantics
// (Cargo.lock:668-679), restated in oracle/ed25519_ref.py.
//
// MI355X design:
//  * one signature per lane, uniform control flow for every lane;
//  * [s]B - [k]A is evaluated as a fixed-base comb with NO doublings:
//        sum_i T_B[i][s_i] + sum_i T_{-A}[i][k_i]
//    with signed radix-2^W digits and per-position tables of affine Niels
//    points j * 2^(W*i) * P, j in [0, 2^(W-1)] (entry 0 = identity).  The B table
//    is built once per context, the -A tables once per signer key (PBFT has a
//    fixed replica set), both resident in HBM and served from L2 / MALL;
//  * R is never decompressed: R' = [s]B - [k]A is compressed (one inversion)
//    and compared with the canonicalised R encoding.  This is equivalent to
//    dalek's point equality R' == decompress(R) ("R check"), and the
//    small-order test on R reduces to a test on y(R') once they are equal.
#pragma once
#include "ge25519.h"
#include "inv25519.h"
#include "sc25519.h"
#include "sha512.h"

#include <type_traits>

namespace pbft {

// Comb table geometry ("plan") over the 254 bits a signed-digit recoding of a
// scalar < 2^253 needs: P positions, the first NB with windows of W+1 bits, the
// rest W bits (P*W + NB >= 254; balanced plans use exactly 254).  Position pos
// starts at bit bitoff(pos) and holds entries j * 2^bitoff(pos) * P0 for
// j = 0 .. 2^(width-1) (entry 0 = identity) at entry offset(pos) of the table.
template <int P_, int W_, int NB_ = 0>
struct plan {
  static_assert(P_ * W_ + NB_ >= 254 && NB_ <= P_, "windows must cover 254 bits");
  static constexpr int P = P_;
  __host__ __device__ static constexpr int width(int pos) { return pos < NB_ ? W_ + 1 : W_; }
  __host__ __device__ static constexpr uint32_t entries(int pos) { return (1u << (width(pos) - 1)) + 1u; }
  __host__ __device__ static constexpr uint32_t offset(int pos) {
    return pos <= NB_ ? (uint32_t)pos * ((1u << W_) + 1u)
                      : (uint32_t)NB_ * ((1u << W_) + 1u) + (uint32_t)(pos - NB_) * ((1u << (W_ - 1)) + 1u);
  }
  __host__ __device__ static constexpr int bitoff(int pos) {
    return pos <= NB_ ? pos * (W_ + 1) : NB_ * (W_ + 1) + (pos - NB_) * W_;
  }
  static constexpr uint32_t ENTRIES = offset(P_);
  static constexpr int ENTRY_WORDS = 32;  // 30 limbs + 2 pad = 128 B
  static constexpr size_t TABLE_WORDS = (size_t)ENTRIES * ENTRY_WORDS;
};
// uniform windows of W bits: positions P = ceil(254/W), entries 2^(W-1)+1 each
template <int W>
struct comb : plan<(254 + W - 1) / W, W, 0> {
  static constexpr uint32_t E = (1u << (W - 1)) + 1u;
};

// Table entry layout (128 B = 32 words), arranged so that the comb kernels can
// pick (hmx, hpx) or (hpx, hmx) -- the entry or its negation -- by LDS address:
//   words  0..7  hpx[0..7]     words  8..15 hmx[0..7]
//   words 16..17 hpx[8..9]     words 18..19 hmx[8..9]
//   words 20..29 dxy[0..9]     words 30..31 zero
// i.e. hpx and hmx start 32 B apart (low 8 limbs) and 8 B apart (top 2 limbs).
__host__ __device__ constexpr int hpx_word(int i) { return i < 8 ? i : 8 + i; }
__host__ __device__ constexpr int hmx_word(int i) { return i < 8 ? 8 + i : 10 + i; }

FE_FN void store_niels(uint32_t* dst, const niels& n) {
#pragma unroll
  for (int i = 0; i < 10; ++i) { dst[hpx_word(i)] = n.hpx.v[i]; dst[hmx_word(i)] = n.hmx.v[i]; dst[20 + i] = n.dxy.v[i]; }
  dst[30] = 0; dst[31] = 0;
}

FE_FN void niels_from_entry_words(niels& n, const uint32_t w[32]) {
#pragma unroll
  for (int i = 0; i < 10; ++i) { n.hpx.v[i] = w[hpx_word(i)]; n.hmx.v[i] = w[hmx_word(i)]; n.dxy.v[i] = w[20 + i]; }
}

FE_FN void load_niels(niels& n, const uint32_t* src) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint4* s4 = (const uint4*)src;
  uint32_t w[32];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint4 v = s4[q];
    w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
  }
  niels_from_entry_words(n, w);
#else
  niels_from_entry_words(n, src);
#endif
}

// Conditional swap of two limb vectors by a lane mask m (0 or ~0): three
// full-rate VOP2 ops per limb pair.  A per-lane `cond ? a : b` compiles to
// v_cndmask_b32_e32 reading VCC, which issues at ~22 cycles per wave on gfx950
// (tools/microbench/valu_mix.hip, profiles/r01_valu_mix.txt) versus ~2.2 for
// v_xor/v_and; m is made opaque so LLVM cannot turn this back into selects.
FE_FN void fe_cswap_mask(fe& x, fe& y, uint32_t m) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t t = (x.v[i] ^ y.v[i]) & m;
    x.v[i] ^= t;
    y.v[i] ^= t;
  }
}

FE_FN uint32_t lane_mask(bool c) {
  uint32_t m = 0u - (uint32_t)c;
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(m));
#endif
  return m;
}

// r = p + sign * q for a halved affine Niels entry q given as (qa, qb, k):
// (hmx, hpx, dxy) for a positive digit, (hpx, hmx, dxy) for a negative one
// (-q = (-x, y) swaps y+x and y-x and negates d*x*y; the comb kernels select qa
// and qb by LDS address).  7 multiplies (6 without T3, for the last step):
//   a = (Y-X) qa, b = (Y+X) qb, c = T k, D = Z  (each half its usual value)
//   E = b - a, F = D -+ c, G = D +- c, H = b + a
//   X3 = E F, Y3 = G H, Z3 = F G, T3 = E H  (= the usual outputs / 4)
#ifndef PBFT_MADD_V2
#define PBFT_MADD_V2 1
#endif
#ifndef PBFT_CHAIN_MIN_N
// comb_kernel uses the single-chain multiplies (CHAIN) from this batch size.  r03: 2^19 (the per-mad laundering
// asm made the chain form slower on one wave of blocks); r04, with one asm block per column: 2^16 (131k shard
// 0.1878 -> 0.1859 ms, 2^20 unchanged; profiles/r04/ab_column_asm.txt)
#define PBFT_CHAIN_MIN_N (1u << 16)
#endif
// 2p - k per limb for canonical k (the conditional negation of the entry's d*x*y)
FE_FN void fe_cneg_canon(fe& out, const fe& k, uint32_t m) {
  fe nk;
  fe_neg(nk, k);
#pragma unroll
  for (int i = 0; i < 10; ++i) out.v[i] = (k.v[i] & ~m) | (nk.v[i] & m);  // one v_bitop3 per limb
}
template <bool WITH_T = true, bool CHAIN = false>
FE_FN void ge_madd_ab(ge& r, const ge& p, const fe& qa, const fe& qb, const fe& k, bool neg) {
#if PBFT_MADD_V2
  // r02 form below, re-ordered for fewer VALU instructions per step (profiles/r03_step_hist.txt):
  //  * the sign of d*x*y is applied to the (canonical) table limbs, k' = +-k (one v_bitop3 + one v_sub per
  //    limb), so F = D - c and G = D + c never swap (the swap cost a v_bitop3 + two v_xor per limb);
  //  * the four output products share their 19x-premultiplied operands: X3 = F E, T3 = H E, Y3 = H G,
  //    Z3 = F G -- {E, G} is a vertex cover of the 4-cycle E-F-G-H, so fe_mul_cols premultiplies 2 vectors
  //    (not 3) and doubles the odd limbs of 2 (not 4).
  // Bounds (every 19x operand < 2^32 / 19, every column < 2^64) in tools/limb_bounds.py ("madd v2").
  fe a, b, c, t, kk;
  fe_cneg_canon(kk, k, lane_mask(neg));
  fe_sub(t, p.Y, p.X);
  if constexpr (CHAIN) {
    // The 3 + 4 products as single-chain multiplies (fe_mul_chain: no 64-bit carry adds; -55 VALU per step).
    // r03 (a laundering asm per mad): faster when many blocks per CU overlap (2^20: -1.8 %), slower on a single
    // wave of blocks (131k: +6 %, profiles/r03/ab_chain_mul.txt); r04 (one asm block per column, no hazard
    // s_nop): faster at 131k too (-1.0 %), so launch_comb_plan uses it from PBFT_CHAIN_MIN_N = 2^16.
    fe t2;
    fe_add(t2, p.Y, p.X);
    {
      fe* const ho[3] = {&a, &b, &c};
      const fe* const fo[3] = {&t, &t2, &p.T};
      const fe* const go[3] = {&qa, &qb, &kk};
      fe_mul_chain<3>(ho, fo, go);
    }
  } else {
    fe_mul(a, t, qa);
    fe_add(t, p.Y, p.X);
    fe_mul(b, t, qb);
    fe_mul(c, p.T, kk);
  }
  fe e, f, g, h;
  fe_sub(e, b, a);
  fe_sub(f, p.Z, c);
  fe_add(g, p.Z, c);
  fe_add(h, b, a);
  if constexpr (CHAIN && WITH_T) {
    fe* const ho[4] = {&r.X, &r.Y, &r.Z, &r.T};
    const fe* const fo[4] = {&f, &h, &f, &h};
    const fe* const go[4] = {&e, &g, &g, &e};
    fe_mul_chain<4>(ho, fo, go);
  } else if constexpr (CHAIN) {
    fe* const ho[3] = {&r.X, &r.Y, &r.Z};
    const fe* const fo[3] = {&f, &h, &f};
    const fe* const go[3] = {&e, &g, &g};
    fe_mul_chain<3>(ho, fo, go);
  } else {
    fe_mul(r.X, f, e);
    fe_mul(r.Y, h, g);
    fe_mul(r.Z, f, g);
    if constexpr (WITH_T) fe_mul(r.T, h, e);
  }
#else
  fe a, b, c, t;
  const uint32_t m = lane_mask(neg);
  fe_sub(t, p.Y, p.X);
  fe_mul(a, t, qa);
  fe_add(t, p.Y, p.X);
  fe_mul(b, t, qb);
  fe_mul(c, p.T, k);
  fe e, f, g, h, dmc, dpc;
  fe_sub(e, b, a);
  fe_sub(dmc, p.Z, c);
  fe_add(dpc, p.Z, c);
  f = dmc;
  g = dpc;
  fe_cswap_mask(f, g, m);
  fe_add(h, b, a);
  // Operand order keeps the 19-premultiplied (second) operand within u32 for
  // either sign: D - c is always a first operand.  Z3 = F*G is dmc*dpc whatever
  // the sign.  Checked by tools/limb_bounds.py.
  fe_mul(r.X, f, e);
  fe_mul(r.Y, g, h);
  fe_mul(r.Z, dmc, dpc);
  if constexpr (WITH_T) fe_mul(r.T, e, h);
#endif
}

// r = p + sign * q, entry q as stored (the swap by masks)
FE_FN void ge_madd_signed(ge& r, const ge& p, const niels& q, bool neg) {
  fe qa = q.hmx, qb = q.hpx;
  fe_cswap_mask(qa, qb, lane_mask(neg));
  ge_madd_ab<true>(r, p, qa, qb, q.dxy, neg);
}

// P = +-q for a halved affine Niels entry given as (qa, qb, k) (see ge_madd_ab),
// as the extended point (x : y : 1 : xy) -- the first comb step costs one
// multiplication (xy = dxy / d) instead of the 7 of a mixed addition to the
// identity.  -q = (-x, y).  The identity entry (1/2, 1/2, 0) gives (0 : 1 : 1 : 0).
// Every output limb vector is carried.
FE_FN void fe_const_dinv(fe& h) {
  const uint32_t w[8] = {0xcdc9f843u, 0x25e0f276u, 0x4279542eu, 0x0b5dd698u,
                         0xcdb9cf66u, 0x2b162114u, 0x14d5ce43u, 0x40907ed2u};
  fe_from_words(h, w);
}
FE_FN void ge_from_ab(ge& P, const fe& qa, const fe& qb, const fe& k, bool neg) {
  const uint32_t m = lane_mask(neg);
  fe_sub(P.X, qb, qa);  // +-x (table limbs are canonical, so qa is carried)
  fe_add(P.Y, qa, qb);  // y
  fe_carry(P.X);
  fe_carry(P.Y);
  fe dinv, t, nt;
  fe_const_dinv(dinv);
  fe_mul(t, k, dinv);  // xy
  fe_neg(nt, t);
  fe_carry(nt);
#pragma unroll
  for (int i = 0; i < 10; ++i) P.T.v[i] = (t.v[i] & ~m) | (nt.v[i] & m);
  fe_one(P.Z);
}
FE_FN void ge_from_niels_signed(ge& P, const niels& q, bool neg) {
  fe qa = q.hmx, qb = q.hpx;
  fe_cswap_mask(qa, qb, lane_mask(neg));
  ge_from_ab(P, qa, qb, q.dxy, neg);
}

// Signed-digit stream over a scalar < 2^253 held in 8 words, one window at a
// time from the bottom: take<W>() returns the next W-bit window's digit in
// [-2^(W-1), 2^(W-1)) and carries; take_last<W>() returns the top window's
// digit without recoding, in [0, 2^(W-1)] (the scalar's bit 253 is 0, so the
// top window plus the incoming carry never exceeds that: every table has the
// entry 2^(W-1)).  Digit i of a plan is the take at width(i) (take_last at P-1).
struct digits {
  uint32_t w[8];
  uint32_t carry;
  FE_FN void init(const uint32_t s[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = s[i];
    carry = 0;
  }
  template <int W>
  FE_FN int take() {
    const uint32_t mask = (1u << W) - 1u;
    int d = (int)((w[0] & mask) + carry);
#pragma unroll
    for (int i = 0; i < 7; ++i) w[i] = (w[i] >> W) | (w[i + 1] << (32 - W));
    w[7] >>= W;
    carry = (d >= (1 << (W - 1))) ? 1u : 0u;
    return d - (int)(carry << W);
  }
  template <int W>
  FE_FN int take_last() {
    return (int)((w[0] & ((1u << W) - 1u)) + carry);
  }
  // the digit of position pos of plan PL (positions taken in order)
  template <class PL, int pos>
  FE_FN int take_pos() {
    if constexpr (pos == PL::P - 1) return take_last<PL::width(pos)>();
    else return take<PL::width(pos)>();
  }
};

// The comb recodes s into table indices, and `digits` assumes s < 2^253 (the
// top digit indexes the last position's table directly).  An attacker-supplied
// s >= L is rejected by check_scalar anyway, but its digits would index past
// the end of the base-point table (bit 253..255 set: up to 2^(W+2) entries too
// far).  So a rejected s is replaced by 0 before recoding: the lane's result
// is already decided (bit 0) and every gather stays inside the table.
FE_FN void sc_clamp_rejected(uint32_t s[8], bool s_ok) {
  const uint32_t m = 0u - (uint32_t)s_ok;
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] &= m;
}

// y in {0, 1, p-1, y8, p-y8}: the y-coordinates of the 8 small-order points.
FE_FN bool y_is_small_order(const uint32_t y[8]) {
  const uint32_t Y8A[8] = {0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u,
                           0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x05fc536du};
  const uint32_t Y8B[8] = {0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du,
                           0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0x7a03ac92u};
  bool z = true, one = true, m1 = true, a8 = true, b8 = true;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    z = z && y[i] == 0u;
    one = one && y[i] == (i == 0 ? 1u : 0u);
    m1 = m1 && y[i] == (i == 0 ? 0xffffffecu : (i == 7 ? 0x7fffffffu : 0xffffffffu));
    a8 = a8 && y[i] == Y8A[i];
    b8 = b8 && y[i] == Y8B[i];
  }
  return z || one || m1 || a8 || b8;
}

// Canonical y of an encoding (bit 255 cleared, minus p when y >= p).
FE_FN void canon_y(uint32_t y[8], const uint32_t enc[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) y[i] = enc[i];
  y[7] &= 0x7fffffffu;
  // y >= p  <=>  y[7] == 0x7fffffff, y[1..6] all ones, y[0] >= 0xffffffed
  bool ge = y[7] == 0x7fffffffu && y[0] >= 0xffffffedu;
#pragma unroll
  for (int i = 1; i < 7; ++i) ge = ge && y[i] == 0xffffffffu;
  if (ge) {
    y[0] -= 0xffffffedu;
#pragma unroll
    for (int i = 1; i < 8; ++i) y[i] = 0;
  }
}

// Compile-time loop: f(std::integral_constant<int, i>) for i = 0 .. N-1.
template <int N, int I = 0, class F>
FE_FN void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>());
    static_for<N, I + 1>(f);
  }
}

// The complete per-lane check.  PLB / PLA: plans of the B table and of this
// lane's -A table; a_enc: raw key encoding (hashed as given).
template <class PLB, class PLA, int LEN>
FE_FN bool verify_lane(const uint32_t r_enc[8], const uint32_t s[8], const uint32_t a_enc[8], bool key_ok,
                       const uint8_t* msg, int len, const uint32_t* tabB, const uint32_t* tabA) {
  const bool s_ok = sc_lt_L(s);
  uint32_t h[16], k[8];
  sha512_ram<LEN>(h, r_enc, a_enc, msg, len);
  sc_reduce512(k, h);

  ge P;
  digits ds, dk;
  uint32_t sc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) sc[i] = s[i];
  sc_clamp_rejected(sc, s_ok);  // rejected s: recode 0 (no gather past the table)
  ds.init(sc);
  dk.init(k);
  constexpr int PB = PLB::P, PA = PLA::P;
  static_for<(PB > PA ? PB : PA)>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    if constexpr (i < PB) {
      const int d = ds.template take_pos<PLB, i>();
      const int ad = d < 0 ? -d : d;
      niels q;
      load_niels(q, tabB + ((size_t)PLB::offset(i) + ad) * 32);
      if (i == 0) ge_from_niels_signed(P, q, d < 0);  // first step: no addition
      else ge_madd_signed(P, P, q, d < 0);
    }
    if constexpr (i < PA) {
      const int d = dk.template take_pos<PLA, i>();
      const int ad = d < 0 ? -d : d;
      niels q;
      load_niels(q, tabA + ((size_t)PLA::offset(i) + ad) * 32);
      ge_madd_signed(P, P, q, d < 0);
    }
  });

  fe zi, x, y;
  fe_invert_gcd(zi, P.Z);
  fe_mul(x, P.X, zi);
  fe_mul(y, P.Y, zi);
  uint32_t xw[8], yw[8], ry[8];
  fe_to_words(xw, x);
  fe_to_words(yw, y);
  canon_y(ry, r_enc);
  bool eq = (xw[0] & 1u) == (r_enc[7] >> 31);
#pragma unroll
  for (int i = 0; i < 8; ++i) eq = eq && yw[i] == ry[i];
  return s_ok && key_ok && eq && !y_is_small_order(yw);
}

// [k]B for k < 2^253 with the base-point comb table of plan PL (RFC 8032 signing side).
template <class PL>
FE_FN void comb_mul_base(ge& P, const uint32_t k[8], const uint32_t* tabB) {
  digits ds;
  ds.init(k);
  static_for<PL::P>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    const int d = ds.template take_pos<PL, i>();
    const int ad = d < 0 ? -d : d;
    niels q;
    load_niels(q, tabB + ((size_t)PL::offset(i) + ad) * 32);
    if (i == 0) ge_from_niels_signed(P, q, d < 0);
    else ge_madd_signed(P, P, q, d < 0);
  });
}

FE_FN void ge_compress_words(uint32_t enc[8], const ge& P) {
  fe zi, x, y;
  fe_invert_gcd(zi, P.Z);
  fe_mul(x, P.X, zi);
  fe_mul(y, P.Y, zi);
  uint32_t xw[8];
  fe_to_words(xw, x);
  fe_to_words(enc, y);
  enc[7] |= (xw[0] & 1u) << 31;
}

// RFC 8032 Ed25519 signature of M under secret seed (8 LE words).
// Outputs R and S encodings (8 LE words each) and the public key A.
template <class PL, int LEN>
FE_FN void sign_lane(uint32_t r_out[8], uint32_t s_out[8], uint32_t a_out[8], const uint32_t seed[8],
                     const uint8_t* msg, int len, const uint32_t* tabB) {
  uint32_t h[16];
  sha512_pre<32, 0>(h, seed, nullptr, 0);           // SHA-512(seed)
  uint32_t a[8], prefix[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { a[i] = h[i]; prefix[i] = h[8 + i]; }
  a[0] &= 0xfffffff8u;                              // clamp
  a[7] &= 0x7fffffffu;
  a[7] |= 0x40000000u;
  uint32_t wide[16], ared[8];
#pragma unroll
  for (int i = 0; i < 16; ++i) wide[i] = i < 8 ? a[i] : 0u;
  sc_reduce512(ared, wide);                         // [a]B = [a mod L]B
  ge P;
  comb_mul_base<PL>(P, ared, tabB);
  ge_compress_words(a_out, P);
  uint32_t rh[16], r[8];
  sha512_pre<32, LEN>(rh, prefix, msg, len);        // r = SHA-512(prefix || M) mod L
  sc_reduce512(r, rh);
  comb_mul_base<PL>(P, r, tabB);
  ge_compress_words(r_out, P);
  uint32_t kh[16], k[8];
  sha512_ram<LEN>(kh, r_out, a_out, msg, len);      // k = SHA-512(R || A || M) mod L
  sc_reduce512(k, kh);
  sc_muladd(s_out, k, a, r);                        // S = (r + k*a) mod L
}

// Table entry (pos, j) of plan PL for base point P0: j * 2^bitoff(pos) * P0.
template <class PL>
FE_FN void comb_entry(niels& out, const ge& P0, int pos, int j) {
  if (j == 0) { niels_identity(out); return; }
  ge Q = P0;
  for (int i = 0; i < PL::bitoff(pos); ++i) ge_dbl(Q, Q);
  ge acc;
  ge_identity(acc);
  bool started = false;
  for (int b = 31; b >= 0; --b) {
    if (started) ge_dbl(acc, acc);
    if ((j >> b) & 1) {
      if (started) { ge t; ge_add(t, acc, Q); acc = t; }
      else { acc = Q; started = true; }
    }
  }
  ge_to_niels(out, acc);
}

}  // namespace pbft
