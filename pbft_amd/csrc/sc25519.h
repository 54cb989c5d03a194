// Scalars mod L = 2^252 + 27742317777372353535851937790883648493, one per lane.
//
//  * sc_lt_L           : ed25519-dalek 1.0.1 check_scalar (reject s >= L)
//  * sc_reduce512      : curve25519-dalek 3.2.1 Scalar::from_hash
//                        (64-byte digest, little-endian, reduced mod L) by
//                        folding 2^252 = -delta in radix 2^21 (sc_reduce512_fold);
//                        Barrett in radix 2^32 (HAC 14.42, k = 8) kept for A/B
//  * sc_muladd         : (a*b + c) mod L, RFC 8032 signing (s = r + k*a)
// Cargo.lock:604-614 (curve25519-dalek), :668-679 (ed25519-dalek).
#pragma once
#include "fe25519.h"

namespace pbft {

#define SC_L_WORDS {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0u, 0u, 0u, 0x10000000u}
// mu = floor(2^512 / L)
#define SC_MU_WORDS {0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du, 0xffffffebu, \
                     0xffffffffu, 0xffffffffu, 0xffffffffu, 0x0000000fu}

// true iff s < L (s: 8 LE words)
FE_FN bool sc_lt_L(const uint32_t s[8]) {
  const uint32_t Lw[8] = SC_L_WORDS;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t d = (uint64_t)s[i] - Lw[i] - borrow;
    borrow = (uint32_t)(d >> 63);
  }
  return borrow != 0;
}

// out[NA+NB] = a[NA] * b[NB]  (product scanning, 96-bit column accumulator)
template <int NA, int NB, int NOUT>
FE_FN void mp_mul(uint32_t out[NOUT], const uint32_t a[NA], const uint32_t b[NB]) {
  uint64_t acc = 0;
  uint32_t acc2 = 0;
#pragma unroll
  for (int c = 0; c < NOUT; ++c) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int j = c - i;
      if (j >= 0 && j < NB) {
        const uint64_t p = (uint64_t)a[i] * b[j];
        acc += p;
        acc2 += (acc < p) ? 1u : 0u;
      }
    }
    out[c] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)acc2 << 32);
    acc2 = 0;
  }
}

// r (9 words) -= L while r >= L (at most twice for Barrett)
FE_FN void sc_cond_sub_L(uint32_t r[9]) {
  const uint32_t Lw[9] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0u, 0u, 0u, 0x10000000u, 0u};
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    uint32_t t[9];
    uint32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const uint64_t d = (uint64_t)r[i] - Lw[i] - borrow;
      t[i] = (uint32_t)d;
      borrow = (uint32_t)(d >> 63);
    }
    const bool ge = borrow == 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) r[i] = ge ? t[i] : r[i];
  }
}

// x: 16 LE words (a 512-bit little-endian integer); out: x mod L, 8 LE words (Barrett; A/B of the fold below)
FE_FN void sc_reduce512_barrett(uint32_t out[8], const uint32_t x[16]) {
  const uint32_t mu[9] = SC_MU_WORDS;
  const uint32_t Lw[8] = SC_L_WORDS;
  uint32_t q1[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) q1[i] = x[7 + i];
  uint32_t q2[18];
  mp_mul<9, 9, 18>(q2, q1, mu);
  uint32_t q3[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) q3[i] = q2[9 + i];
  uint32_t r2[9];
  mp_mul<9, 8, 9>(r2, q3, Lw);
  uint32_t r[9];
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint64_t d = (uint64_t)x[i] - r2[i] - borrow;
    r[i] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
  // r1 - r2 mod 2^288 is already correct (the wrap is implicit)
  sc_cond_sub_L(r);
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = r[i];
}

// x mod L by folding, for the verifier's challenge scalar (the same value as sc_reduce512).
// 2^252 = -delta (mod L), delta = L - 2^252 < 2^125, and 252 = 12 x 21: the 512-bit input as 25 signed
// limbs of radix 2^21; every limb at or above 2^252 is multiplied by the signed radix-2^21 digits of -delta
// (|digit| < 2^20) and added 12 limbs lower.  Signed carries between the folds keep every multiplied limb
// inside int32 (one v_mad_i64_i32 per product, 90 in all) and every column below 2^50; no 96-bit
// accumulators and no compare-and-select carries as in the Barrett form.  Bounds: after the fold of limbs
// 18..24 the limbs 6..16 are < 2^43.6, carried to [-2^20, 2^20) (limb 17 < 2^28.2); after the fold of
// 12..17 limbs 0..11 are < 2^49; two more folds of limb 12 (< 2^8, then a carry of +-2) and floor carries
// leave limbs 0..10 in [0, 2^21) and |limb 11| <= 2^20 + 2, so v = sum < 2^252 < L and v > -2^251 > -L:
// one conditional +L gives the canonical residue.  Host harness: test_reduce512 (3,000 random 512-bit values
// and edge cases vs Python).
FE_FN void sc_reduce512_fold(uint32_t out[8], const uint32_t x[16]) {
  const int32_t C[6] = {666643, 470296, 654183, -997805, 136657, -683901};  // -delta, signed radix 2^21
  int64_t s[25];
#pragma unroll
  for (int i = 0; i < 24; ++i) {
    const int b = 21 * i, q = b >> 5, sh = b & 31;
    const uint64_t v = ((uint64_t)(q + 1 < 16 ? x[q + 1] : 0u) << 32) | x[q];
    s[i] = (int64_t)((v >> sh) & 0x1FFFFFu);
  }
  s[24] = (int64_t)(x[15] >> 24);
  auto fold = [&](int i) {
    const int32_t si = (int32_t)s[i];
#pragma unroll
    for (int j = 0; j < 6; ++j) s[i - 12 + j] += (int64_t)si * C[j];
    s[i] = 0;
  };
  auto carry = [&](int i) {  // signed, rounding: s[i] into [-2^20, 2^20)
    const int64_t c = (s[i] + (1 << 20)) >> 21;
    s[i + 1] += c;
    s[i] -= c * (1 << 21);
  };
#pragma unroll
  for (int i = 24; i >= 18; --i) fold(i);
#pragma unroll
  for (int i = 6; i <= 16; ++i) carry(i);
#pragma unroll
  for (int i = 17; i >= 12; --i) fold(i);
#pragma unroll
  for (int i = 0; i <= 11; ++i) carry(i);
  fold(12);
#pragma unroll
  for (int i = 0; i <= 11; ++i) carry(i);
  fold(12);
#pragma unroll
  for (int i = 0; i <= 10; ++i) {  // floor carries: limbs 0..10 in [0, 2^21)
    const int64_t c = s[i] >> 21;
    s[i + 1] += c;
    s[i] -= c * (1 << 21);
  }
  // pack limbs 0..10 (231 bits) + limb 11 * 2^231 into a 288-bit two's complement value
  uint32_t w[9];
  uint64_t acc = 0;
  int nb = 0, k = 0;
#pragma unroll
  for (int i = 0; i <= 10; ++i) {
    acc |= (uint64_t)s[i] << nb;
    nb += 21;
    if (nb >= 32) { w[k++] = (uint32_t)acc; acc >>= 32; nb -= 32; }
  }
  // k == 7, nb == 7: bits 224..230 in acc
  w[7] = (uint32_t)acc | (uint32_t)((uint64_t)s[11] << 7);
  w[8] = (uint32_t)(s[11] >> 25);
  // negative: + L (then < L)
  const uint32_t Lw[8] = SC_L_WORDS;
  const uint32_t m = 0u - (w[8] >> 31);
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t t = (uint64_t)w[i] + (Lw[i] & m) + c;
    out[i] = (uint32_t)t;
    c = (uint32_t)(t >> 32);
  }
}

#ifndef PBFT_SC_BARRETT
#define PBFT_SC_BARRETT 0
#endif
// x mod L (curve25519-dalek Scalar::from_hash): the fold; PBFT_SC_BARRETT=1 for the Barrett form
FE_FN void sc_reduce512(uint32_t out[8], const uint32_t x[16]) {
#if PBFT_SC_BARRETT
  sc_reduce512_barrett(out, x);
#else
  sc_reduce512_fold(out, x);
#endif
}

// out = (a*b + c) mod L; all 8-word little-endian, a,b,c < 2^256
FE_FN void sc_muladd(uint32_t out[8], const uint32_t a[8], const uint32_t b[8], const uint32_t c[8]) {
  uint32_t p[16];
  mp_mul<8, 8, 16>(p, a, b);
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint64_t s = (uint64_t)p[i] + (i < 8 ? c[i] : 0u) + carry;
    p[i] = (uint32_t)s;
    carry = (uint32_t)(s >> 32);
  }
  // a*b + c < 2^512 since a, b < 2^256 - 2^255 in practice (a < 2^255, b < L)
  sc_reduce512(out, p);
}

}  // namespace pbft
