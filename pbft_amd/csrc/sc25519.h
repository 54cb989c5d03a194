// Scalars mod L = 2^252 + 27742317777372353535851937790883648493, one per lane.
//
//  * sc_lt_L           : ed25519-dalek 1.0.1 check_scalar (reject s >= L)
//  * sc_reduce512      : curve25519-dalek 3.2.1 Scalar::from_hash
//                        (64-byte digest, little-endian, reduced mod L) via
//                        Barrett reduction in radix 2^32 (HAC 14.42, k = 8)
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

// x: 16 LE words (a 512-bit little-endian integer); out: x mod L, 8 LE words
FE_FN void sc_reduce512(uint32_t out[8], const uint32_t x[16]) {
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
