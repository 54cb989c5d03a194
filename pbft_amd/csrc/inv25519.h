// Constant-time inversion in GF(2^255 - 19) by Bernstein-Yang divsteps
// ("safegcd", half-delta variant), one field element per lane, 32-bit VALU.
//
// Why: the verifier's only inversions (batch-inversion finish, latency-mode
// compare, table build) are latency-bound serial chains -- one wave per SIMD
// walking z^(p-2), 254 squarings + 11 multiplications of ~165 instructions
// each (~44k instructions, ~80-130 us on MI355X).  Divsteps on 30-bit limbs
// need ~19k instructions whose dependency chain is mostly 32-bit VOP2 work.
//
// Algorithm (Bernstein & Yang, "Fast constant-time gcd computation and modular
// inversion", 2019; half-delta divsteps with zeta = -(delta + 1/2)): 20 batches
// of 30 divsteps = 600 >= 590, the divstep bound for 256-bit inputs.  Each
// batch runs the divsteps on the low 30 bits of f and g, producing a 2x2
// transition matrix t with 2^30 [f', g'] = t [f, g]; t is then applied to the
// full-width f, g (exactly divisible by 2^30) and to d, e modulo p (d, e are
// kept in (-2p, p); a multiple of p is added so that the low 30 bits vanish).
// Invariants f = d x, g = e x (mod p); at the end f = +-1 and x^-1 = +-d.
// x = 0 yields 0 (like z^(p-2)).  Checked against fe_invert (z^(p-2)) in the
// host harness (tests/test_host_harness.py) and on the GPU.
#pragma once
#include "fe25519.h"

namespace pbft {

struct s30 {
  int32_t v[9];  // sum v[i] 2^(30 i); v[0..7] in [0, 2^30) between batches, v[8] signed
};

#define INV_M30 0x3FFFFFFFu
#define INV_PINV30 0x179435E5u  // p^-1 mod 2^30

__host__ __device__ __forceinline__ int32_t p30_limb(int i) {
  return i == 0 ? 0x3FFFFFED : (i == 8 ? 0x7FFF : 0x3FFFFFFF);
}

// 30 half-delta divsteps on the low bits of f and g (uniform control flow).
// Returns the new zeta; t = {u, v, q, r} with 2^30 f' = u f + v g, 2^30 g' = q f + r g.
__host__ __device__ __forceinline__ int32_t divsteps30(int32_t zeta, uint32_t f, uint32_t g, int32_t t[4]) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll
  for (int i = 0; i < 30; ++i) {
    const uint32_t c1 = (uint32_t)(zeta >> 31);  // zeta < 0
    const uint32_t c2 = 0u - (g & 1u);           // g odd
    // zeta < 0 and g odd: swap (f <- old g) and zeta <- -zeta - 2; else zeta <- zeta - 1
    const uint32_t c3 = c1 & c2;
    const uint32_t n3 = c3 >> 31;                // -c3 (0 or 1)
    // g odd: g += f (zeta >= 0) or g -= f (zeta < 0), and the same on the g row of t.
    // ((x ^ c1) - c1) & c2 == ((x ^ c1) & c2) - c3: one v_bitop3 + one v_add3 per row
    // (18 VALU per divstep instead of 23 -- the chain of every inversion)
    g = g + ((f ^ c1) & c2) + n3;
    q = q + ((u ^ c1) & c2) + n3;
    r = r + ((v ^ c1) & c2) + n3;
    zeta = (zeta ^ (int32_t)c3) - 1;
    f += g & c3;
    u = (u + (q & c3)) << 1;
    v = (v + (r & c3)) << 1;
    g >>= 1;
  }
  t[0] = (int32_t)u; t[1] = (int32_t)v; t[2] = (int32_t)q; t[3] = (int32_t)r;
  return zeta;
}

// [f, g] <- t [f, g] / 2^30 (exact)
__host__ __device__ __forceinline__ void inv_update_fg(s30& f, s30& g, const int32_t t[4]) {
  const int64_t u = t[0], v = t[1], q = t[2], r = t[3];
  int64_t cf = u * f.v[0] + v * g.v[0];
  int64_t cg = q * f.v[0] + r * g.v[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 9; ++i) {
    cf += u * f.v[i] + v * g.v[i];
    cg += q * f.v[i] + r * g.v[i];
    f.v[i - 1] = (int32_t)((uint32_t)cf & INV_M30);
    g.v[i - 1] = (int32_t)((uint32_t)cg & INV_M30);
    cf >>= 30;
    cg >>= 30;
  }
  f.v[8] = (int32_t)cf;
  g.v[8] = (int32_t)cg;
}

// [d, e] <- (t [d, e] + p [md, me]) / 2^30, md, me chosen so the division is exact
// and d, e stay in (-2p, p).
__host__ __device__ __forceinline__ void inv_update_de(s30& d, s30& e, const int32_t t[4]) {
  const int64_t u = t[0], v = t[1], q = t[2], r = t[3];
  const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;  // d < 0, e < 0
  int32_t md = (t[0] & sd) + (t[1] & se);
  int32_t me = (t[2] & sd) + (t[3] & se);
  int64_t cd = u * d.v[0] + v * e.v[0];
  int64_t ce = q * d.v[0] + r * e.v[0];
  md -= (int32_t)((INV_PINV30 * (uint32_t)cd + (uint32_t)md) & INV_M30);
  me -= (int32_t)((INV_PINV30 * (uint32_t)ce + (uint32_t)me) & INV_M30);
  cd += (int64_t)p30_limb(0) * md;
  ce += (int64_t)p30_limb(0) * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 9; ++i) {
    cd += u * d.v[i] + v * e.v[i] + (int64_t)p30_limb(i) * md;
    ce += q * d.v[i] + r * e.v[i] + (int64_t)p30_limb(i) * me;
    d.v[i - 1] = (int32_t)((uint32_t)cd & INV_M30);
    e.v[i - 1] = (int32_t)((uint32_t)ce & INV_M30);
    cd >>= 30;
    ce >>= 30;
  }
  d.v[8] = (int32_t)cd;
  e.v[8] = (int32_t)ce;
}

// propagate limb carries (limbs may be any int32 after an add / negate)
__host__ __device__ __forceinline__ void inv_carry(s30& r) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    r.v[i + 1] += r.v[i] >> 30;
    r.v[i] = (int32_t)((uint32_t)r.v[i] & INV_M30);
  }
}

// r in (-2p, p), neg_mask = -1 if the result must be negated: r <- +-r mod p in [0, p)
__host__ __device__ __forceinline__ void inv_normalize(s30& r, int32_t neg_mask) {
  int32_t c = r.v[8] >> 31;  // r < 0: add p
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = ((r.v[i] + (p30_limb(i) & c)) ^ neg_mask) - neg_mask;
  inv_carry(r);
  c = r.v[8] >> 31;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] += p30_limb(i) & c;
  inv_carry(r);
}

// out = z^-1 (0 -> 0); z any fe (carried or one add/sub away from carried)
__host__ __device__ __forceinline__ void fe_invert_gcd(fe& out, const fe& z) {
  uint32_t w[8];
  fe_to_words(w, z);  // canonical, < p
  s30 f, g, d, e;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int b = 30 * i, wi = b >> 5, sh = b & 31;
    uint64_t x = w[wi] >> sh;
    if (wi + 1 < 8) x |= (uint64_t)w[wi + 1] << (32 - sh);
    g.v[i] = (int32_t)((uint32_t)x & INV_M30);
    f.v[i] = p30_limb(i);
    d.v[i] = 0;
    e.v[i] = i == 0 ? 1 : 0;
  }
  int32_t zeta = -1;
#pragma nounroll
  for (int it = 0; it < 20; ++it) {
    int32_t t[4];
    zeta = divsteps30(zeta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    inv_update_de(d, e, t);
    inv_update_fg(f, g, t);
  }
  inv_normalize(d, f.v[8] >> 31);  // f = +-1
  // 30-bit limbs -> 8 little-endian words -> radix 2^25.5 limbs
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int b = 32 * j, li = b / 30, sh = b % 30;
    uint64_t x = (uint64_t)(uint32_t)d.v[li] >> sh;
    x |= (uint64_t)(uint32_t)d.v[li + 1] << (30 - sh);
    if (li + 2 < 9 && 60 - sh < 32) x |= (uint64_t)(uint32_t)d.v[li + 2] << (60 - sh);
    w[j] = (uint32_t)x;
  }
  fe_from_words(out, w);
}

// ---- variable-time form, for a wave-UNIFORM input --------------------------------
// The finish kernel's cross-lane product tree leaves the same value in every lane
// of a wave, so data-dependent branches never diverge and the public value needs
// no constant-time treatment.  Original-delta divsteps (eta = -delta, starting at
// -1; Bernstein & Yang 2019, the variable-time batching of libsecp256k1's
// modinv32_var): the zeros of g are shifted out at once (ctz) and, while no swap
// can occur (eta >= 0), up to min(eta + 1, steps left, 20) low bits of g are
// cleared in ONE step g += w f with w = -g / f mod 2^limit (f^-1 mod 2^20 by
// Newton's iteration from (3 f) ^ 2, exact to 5 bits).  The batch ends after 30
// divsteps with the same transition-matrix convention as divsteps30 (2^30 f' =
// u f + v g, 2^30 g' = q f + r g), so inv_update_de / inv_update_fg apply
// unchanged; batches run until g = 0 (at most 25: the 724-divstep bound for
// 256-bit inputs), then f = +-1 and x^-1 = +-d.  The inverse is unique, so the
// result is bit-identical to fe_invert_gcd / z^(p-2).
__host__ __device__ __forceinline__ int32_t divsteps30_var(int32_t eta, uint32_t f, uint32_t g, int32_t t[4]) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  int i = 30;
  for (;;) {
    const int zeros = __builtin_ctz(g | (0xFFFFFFFFu << i));  // i >= 1: the mask has a set bit
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    // f and g odd
    if (eta < 0) {  // delta > 0: swap (f, g) <- (g, -f), rows alike
      eta = -eta;
      uint32_t x = f; f = g; g = 0u - x;
      x = u; u = q; q = 0u - x;
      x = v; v = r; r = 0u - x;
    }
    int limit = eta + 1 < i ? eta + 1 : i;
    if (limit > 20) limit = 20;
    const uint32_t m = 0xFFFFFFFFu >> (32 - limit);
    uint32_t y = (3u * f) ^ 2u;  // f^-1 mod 2^5
    y *= 2u - f * y;             // mod 2^10
    y *= 2u - f * y;             // mod 2^20
    const uint32_t w = (0u - g * y) & m;  // g + w f = 0 mod 2^limit
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t[0] = (int32_t)u; t[1] = (int32_t)v; t[2] = (int32_t)q; t[3] = (int32_t)r;
  return eta;
}

// out = z^-1 (0 -> 0) for a wave-uniform z (see above); z as for fe_invert_gcd
// (The scalar unit does not help here, measured r03 with PBFT_FIN_STAMPS: run on the SALU, the divsteps take
// half their VALU time but the 30-bit-limb updates, which need 64-bit products, take as long as the divsteps
// saved -- whole-inversion or hybrid alike, ~78k shader cycles either way; profiles/r03/finish_stamps.txt.)
__host__ __device__ __forceinline__ void fe_invert_var(fe& out, const fe& z, uint64_t* prof = nullptr) {
  uint32_t w[8];
  fe_to_words(w, z);
  s30 f, g, d, e;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int b = 30 * i, wi = b >> 5, sh = b & 31;
    uint64_t x = w[wi] >> sh;
    if (wi + 1 < 8) x |= (uint64_t)w[wi + 1] << (32 - sh);
    g.v[i] = (int32_t)((uint32_t)x & INV_M30);
    f.v[i] = p30_limb(i);
    d.v[i] = 0;
    e.v[i] = i == 0 ? 1 : 0;
  }
  int32_t eta = -1;
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t t_ds = 0, t_up = 0, n_it = 0;
#endif
  for (int it = 0; it < 25; ++it) {
    int32_t nz = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) nz |= g.v[i];
    if (nz == 0) break;
    int32_t t[4];
#if defined(__HIP_DEVICE_COMPILE__)
    uint64_t c0 = 0, c1 = 0;
    if (prof) c0 = __builtin_amdgcn_s_memtime();
#endif
    eta = divsteps30_var(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
#if defined(__HIP_DEVICE_COMPILE__)
    if (prof) { asm volatile("" :: "v"(t[0]), "v"(t[3])); c1 = __builtin_amdgcn_s_memtime(); t_ds += c1 - c0; }
#endif
    inv_update_de(d, e, t);
    inv_update_fg(f, g, t);
#if defined(__HIP_DEVICE_COMPILE__)
    if (prof) {
      asm volatile("" :: "v"(f.v[0]), "v"(g.v[0]), "v"(d.v[8]), "v"(e.v[8]));
      t_up += __builtin_amdgcn_s_memtime() - c1;
      ++n_it;
    }
#endif
  }
#if defined(__HIP_DEVICE_COMPILE__)
  if (prof) { prof[0] = t_ds; prof[1] = t_up; prof[2] = n_it; }
#endif
  inv_normalize(d, f.v[8] >> 31);  // f = +-1
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int b = 32 * j, li = b / 30, sh = b % 30;
    uint64_t x = (uint64_t)(uint32_t)d.v[li] >> sh;
    x |= (uint64_t)(uint32_t)d.v[li + 1] << (30 - sh);
    if (li + 2 < 9 && 60 - sh < 32) x |= (uint64_t)(uint32_t)d.v[li + 2] << (60 - sh);
    w[j] = (uint32_t)x;
  }
  fe_from_words(out, w);
}

}  // namespace pbft
