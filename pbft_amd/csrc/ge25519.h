// Edwards25519 group operations for gfx950 (twisted Edwards, a = -1).
//
// Points live in extended coordinates (X:Y:Z:T), x = X/Z, y = Y/Z, xy = T/Z
// (40 VGPRs).  Table entries are HALVED affine Niels triples ((y+x)/2, (y-x)/2,
// d*x*y), fully reduced: the mixed addition (verify_core.h) then computes every
// product at half the usual value and uses D = Z1 instead of 2*Z1, so its four
// outputs are the usual ones / 4 -- the same projective point, without the
// doubling of Z1 in every comb step.  The unified
// formulas are complete for a = -1 and non-square d, so torsion components
// (mixed-order keys, small-order R) need no special casing -- the same property
// curve25519-dalek 3.2.1 relies on (Cargo.lock:604-614).
#pragma once
#include "fe25519.h"

namespace pbft {

struct ge { fe X, Y, Z, T; };
struct niels { fe hpx, hmx, dxy; };  // (y+x)/2, (y-x)/2, d*x*y

// 2*d and d in radix 2^25.5 (canonical)
FE_FN void fe_const_d(fe& h) {
  const uint32_t w[8] = {0x135978a3u, 0x75eb4dcau, 0x4141d8abu, 0x00700a4du,
                         0x7779e898u, 0x8cc74079u, 0x2b6ffe73u, 0x52036ceeu};
  fe_from_words(h, w);
}
FE_FN void fe_const_2d(fe& h) {
  const uint32_t w[8] = {0x26b2f159u, 0xebd69b94u, 0x8283b156u, 0x00e0149au,
                         0xeef3d130u, 0x198e80f2u, 0x56dffce7u, 0x2406d9dcu};
  fe_from_words(h, w);
}
FE_FN void fe_const_sqrtm1(fe& h) {
  const uint32_t w[8] = {0x4a0ea0b0u, 0xc4ee1b27u, 0xad2fe478u, 0x2f431806u,
                         0x3dfbd7a7u, 0x2b4d0099u, 0x4fc1df0bu, 0x2b832480u};
  fe_from_words(h, w);
}

// 1/2 = (p + 1) / 2 = 2^254 - 9
FE_FN void fe_const_half(fe& h) {
  const uint32_t w[8] = {0xfffffff7u, 0xffffffffu, 0xffffffffu, 0xffffffffu,
                         0xffffffffu, 0xffffffffu, 0xffffffffu, 0x3fffffffu};
  fe_from_words(h, w);
}

FE_FN void ge_identity(ge& p) { fe_zero(p.X); fe_one(p.Y); fe_one(p.Z); fe_zero(p.T); }
FE_FN void niels_identity(niels& n) { fe_const_half(n.hpx); fe_const_half(n.hmx); fe_zero(n.dxy); }

// r = p + q, both extended (8 multiplies; used in table precomputation)
FE_FN void ge_add(ge& r, const ge& p, const ge& q) {
  fe a, b, c, d, t, k;
  fe_sub(t, p.Y, p.X); fe_sub(a, q.Y, q.X); fe_carry(t); fe_carry(a); fe_mul(a, t, a);
  fe_add(t, p.Y, p.X); fe_add(b, q.Y, q.X); fe_mul(b, t, b);
  fe_const_2d(k);
  fe_mul(c, p.T, q.T); fe_mul(c, c, k);
  fe_mul(d, p.Z, q.Z); fe_add(d, d, d);
  fe e, f, g, h;
  fe_sub(e, b, a); fe_sub(f, d, c); fe_add(g, d, c); fe_add(h, b, a);
  fe_carry(e); fe_carry(f); fe_carry(g); fe_carry(h);
  fe_mul(r.X, e, f); fe_mul(r.Y, g, h); fe_mul(r.Z, f, g); fe_mul(r.T, e, h);
}

// r = 2p (dbl-2008-hwcd, a = -1; E, F, G, H carried before the products)
FE_FN void ge_dbl(ge& r, const ge& p) {
  fe a, b, c, e, f, g, h, t;
  fe_sq(a, p.X);
  fe_sq(b, p.Y);
  fe_sq(c, p.Z); fe_add(c, c, c);
  fe_add(t, p.X, p.Y); fe_sq(t, t);
  fe_add(h, a, b); fe_carry(h);   // H' = A + B          (= -H)
  fe_sub(e, h, t); fe_carry(e);   // E' = H' - (X+Y)^2   (= -E)
  fe_sub(g, a, b); fe_carry(g);   // G' = A - B          (= -G)
  fe_carry(c);
  fe_add(f, c, g); fe_carry(f);   // F' = 2Z^2 + G'      (= -F)
  fe_mul(r.X, e, f); fe_mul(r.Y, g, h); fe_mul(r.T, e, h); fe_mul(r.Z, f, g);
}

FE_FN void ge_neg(ge& r, const ge& p) {
  r.Y = p.Y; r.Z = p.Z;
  fe_neg(r.X, p.X); fe_neg(r.T, p.T);
  fe_carry(r.X); fe_carry(r.T);
}

FE_FN bool ge_is_identity(const ge& p) {
  // X == 0 and Y == Z
  return fe_is_zero(p.X) && fe_eq(p.Y, p.Z);
}

FE_FN bool ge_is_small_order(const ge& p) {
  ge q;
  ge_dbl(q, p); ge_dbl(q, q); ge_dbl(q, q);
  return ge_is_identity(q);
}

// curve25519-dalek 3.2.1 CompressedEdwardsY::decompress (y not range-checked;
// x = 0 with sign bit 1 accepted).  w = 8 LE words of the encoding.
template <bool PAR = false>
FE_FN bool ge_decompress(ge& p, const uint32_t w[8]) {
  fe y, one, yy, u, v, v3, v7, r, chk, d, i, nu, nui, t;
  fe_from_words(y, w);
  fe_one(one);
  fe_sq(yy, y);
  fe_sub(u, yy, one); fe_carry(u);
  fe_const_d(d);
  fe_mul(v, yy, d); fe_add(v, v, one);
  fe_sq(v3, v); fe_mul(v3, v3, v);
  fe_sq(v7, v3); fe_mul(v7, v7, v);
  fe_mul(t, u, v7);
  fe_pow22523<PAR>(r, t);
  fe_mul(r, r, u); fe_mul(r, r, v3);
  fe_sq(chk, r); fe_mul(chk, chk, v);
  fe_neg(nu, u); fe_carry(nu);
  fe_const_sqrtm1(i);
  fe_mul(nui, nu, i);
  const bool correct = fe_eq(chk, u), flipped = fe_eq(chk, nu), flipped_i = fe_eq(chk, nui);
  fe ri;
  fe_mul(ri, r, i);
  fe_cmov(r, ri, flipped || flipped_i);
  fe rn;
  fe_neg(rn, r); fe_carry(rn);
  fe_cmov(r, rn, fe_is_negative(r));
  if (w[7] >> 31) { fe_neg(rn, r); fe_carry(rn); r = rn; }
  p.X = r; p.Y = y; fe_one(p.Z); fe_mul(p.T, r, y);
  return correct || flipped;
}

// Halved affine Niels entry of the affine point (x, y), every coordinate canonical
// (so table limbs are minimal).
FE_FN void niels_from_affine(niels& n, const fe& x, const fe& y) {
  fe t, half, d;
  fe_const_half(half);
  fe_const_d(d);
  fe_add(t, y, x);
  fe_mul(n.hpx, t, half);
  fe_sub(t, y, x);
  fe_mul(n.hmx, t, half);
  fe_mul(t, x, y);
  fe_mul(n.dxy, t, d);
  uint32_t w[8];
  fe_to_words(w, n.hpx); fe_from_words(n.hpx, w);
  fe_to_words(w, n.hmx); fe_from_words(n.hmx, w);
  fe_to_words(w, n.dxy); fe_from_words(n.dxy, w);
}

// halved affine Niels form of p (one inversion)
FE_FN void ge_to_niels(niels& n, const ge& p) {
  fe zi, x, y;
  fe_invert(zi, p.Z);
  fe_mul(x, p.X, zi);
  fe_mul(y, p.Y, zi);
  niels_from_affine(n, x, y);
}

}  // namespace pbft
