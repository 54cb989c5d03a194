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

// ---- table-driven divsteps, for a wave-uniform input ------------------------------
// The half-delta divsteps of divsteps30, DS_TN = 5 at a time: the 5 steps' decisions depend only on zeta's
// class (clamp(zeta, -5, 4): from zeta >= 4 no swap can occur within 5 steps, and every zeta <= -5 takes the
// same decisions), f mod 32 (odd) and g mod 32, so one lookup gives their 2x2 transition matrix S
// (2^5 [f'; g'] = S [f; g], entries in [-32, 32]) and the affine map zeta' = +-zeta + c.  A batch of 30 is six
// lookups, T <- S T each, and ends with the same t and zeta as divsteps30 (host-tested step for step), so
// inv_update_de / inv_update_fg apply unchanged.  With the 5,120-entry table in LDS (40 KB) a lookup is one
// ds_read_b64 plus ~8 dependent VALU operations on the critical path instead of ~5 x 18 (constant-time) or
// the ctz / Newton-inverse chain of divsteps30_var.
#define DS_TN 5
#ifndef PBFT_INV_VALU_LOOKUP
#define PBFT_INV_VALU_LOOKUP 1  // the divstep lookups on the VALU (row broadcast): -13 % inversion cycles (profiles/r03/ab_finish.txt)
#endif
#ifndef PBFT_INV_WAVE
#define PBFT_INV_WAVE 1  // wave-uniform inversions: fe_invert_wave (limbs across lanes) instead of fe_invert_tab
#endif
#define DS_TZ (2 * DS_TN)
#define DS_TAB_ENTRIES (DS_TZ * 16 * 32)

// entry idx = ((zc + 5) * 16 + (f >> 1) % 16) * 32 + g % 32, i.e. byte offset 4096 (zc + 5) + 256 ((f >> 1) % 16) +
// 8 (g % 32): u, v, q, r as int8 in the low word; the high word is the zeta map in the scaled form that indexes the
// table, Z = 4096 (zeta + 5): 4096 c when zeta' = zeta + c, 4096 c + 40961 when zeta' = c - zeta, so that
// Z' = (Z ^ -(hi & 1)) + hi (one v_xad_u32 after a one-bit sign extension) and the class's byte offset is
// med3(Z, 0, 9 * 4096).
__host__ __device__ constexpr uint64_t ds_tab_entry(uint32_t idx) {
  int32_t zeta = (int32_t)(idx / 512) - DS_TN;
  int32_t f = (int32_t)((((idx / 32) % 16) << 1) | 1), g = (int32_t)(idx % 32);
  int32_t u = 1, v = 0, q = 0, r = 1, s = 1, c = 0;
  for (int i = 0; i < DS_TN; ++i) {
    const bool c1 = zeta < 0, c2 = (g & 1) != 0, c3 = c1 && c2;
    if (c2) {
      g += c1 ? -f : f;
      q += c1 ? -u : u;
      r += c1 ? -v : v;
    }
    if (c3) { zeta = -zeta - 2; s = -s; c = -c - 2; f += g; u += q; v += r; }
    else { zeta -= 1; c -= 1; }
    u *= 2; v *= 2;
    g /= 2;  // exact: g is even here
  }
  const int32_t hi = s < 0 ? 4096 * c + 40961 : 4096 * c;
  return (uint64_t)(uint8_t)(int8_t)u | (uint64_t)(uint8_t)(int8_t)v << 8 | (uint64_t)(uint8_t)(int8_t)q << 16 |
         (uint64_t)(uint8_t)(int8_t)r << 24 | (uint64_t)(uint32_t)hi << 32;
}
struct ds_table {
  uint64_t e[DS_TAB_ENTRIES];
  constexpr ds_table() : e() {
    for (uint32_t i = 0; i < DS_TAB_ENTRIES; ++i) e[i] = ds_tab_entry(i);
  }
};

// low 24 bits, sign-extended: the operand v_mul_i32_i24 / v_mad_i32_i24 read (the compiler selects them for
// products of such values and drops the extension)
__host__ __device__ __forceinline__ int32_t ds_sext24(uint32_t x) { return (int32_t)(x << 8) >> 8; }

// byte offset of the entry: scaled zeta Z's class, f's bits 1..4 moved to bits 8..11 and g's bits 0..4 to bits 3..7
// by the shifts FS, GS (> 0 left, < 0 right)
template <int FS, int GS>
__host__ __device__ __forceinline__ uint32_t ds_offset(int32_t Z, uint32_t F, uint32_t G) {
  const int32_t zc = Z < 0 ? 0 : (Z > 9 * 4096 ? 9 * 4096 : Z);
  const uint32_t fp = FS >= 0 ? F << (FS & 31) : F >> (-FS & 31);
  const uint32_t gp = GS >= 0 ? G << (GS & 31) : G >> (-GS & 31);
  return (fp & 0xF00u) | (gp & 0xF8u) | (uint32_t)zc;
}

// Schedule pin (device): xs are treated as rewritten after `dep` exists, so work reading them is issued after the
// instruction that produced `dep` -- the lookup chain below issues each ds_read first and fills its latency with
// the independent products (the compiler otherwise interleaves them ahead of the address and the read).
__host__ __device__ __forceinline__ void ds_after1(uint32_t dep, int32_t& x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(x) : "v"(dep));
#else
  (void)dep; (void)x;
#endif
}
template <class... T>
__host__ __device__ __forceinline__ void ds_after(uint32_t dep, T&... xs) {
  (ds_after1(dep, xs), ...);
}

struct ds_mat {
  int32_t u, v, q, r;
};

__host__ __device__ __forceinline__ uint64_t ds_load(const uint64_t* tab, uint32_t off) {
  return *(const uint64_t*)((const char*)tab + off);
}
// lookup 0's offset (its entry e0 = ds_load(tab, off0) is read by the caller, which can issue it early)
__host__ __device__ __forceinline__ uint32_t ds_first(int32_t Z, uint32_t f, uint32_t g) {
  return ds_offset<7, 3>(Z, f, g);
}

// 30 half-delta divsteps by 6 lookups on the scaled zeta Z = 4096 (zeta + 5); t as divsteps30.  The low bits of f
// and g are never shifted: after lookup j they are F = 2^(5j) f_j, G = 2^(5j) g_j (mod 2^30), and lookup j reads
// their bits 5j .. 5j+4 in place.  Lookups 0-2 multiply in 32 bits; from lookup 3 the window F >> 6 (bits 6..29 of
// F, low 10 bits zero) is exact in 24-bit products, as are the matrix products up to T_5 (entries < 2^20 before the
// fifth); the sixth, T_6 = S_5 T_5, is 32-bit.  Per lookup on the chain: the entry's fields, two products, the
// offset, the read; the matrix products T <- S T and fill(k, off) (the caller's independent work) are pinned after
// lookup k's read is issued; lookup 0's entry e0 (at off0) comes from the caller.
template <class Fill>
__host__ __device__ __forceinline__ int32_t divsteps30_tabz(int32_t Z, uint32_t f, uint32_t g, uint32_t off0,
                                                            uint64_t e0, int32_t t[4], const uint64_t* tab,
                                                            Fill&& fill) {
  auto load = [&](uint32_t off) { return ds_load(tab, off); };
  auto decode = [&](uint64_t e) {
    const uint32_t lo = (uint32_t)e;
    const int32_t hi = (int32_t)(e >> 32);
    Z = (int32_t)(((uint32_t)Z ^ (uint32_t)((int32_t)((uint32_t)hi << 31) >> 31)) + (uint32_t)hi);
    return ds_mat{(int8_t)lo, (int8_t)(lo >> 8), (int8_t)(lo >> 16), (int32_t)lo >> 24};
  };
  // products in 32 bits (wrapping) and in 24 bits (the low 24 bits of both operands, sign-extended)
  auto mul32 = [](int32_t s, uint32_t x) { return (uint32_t)s * x; };
  auto mul24 = [](int32_t s, uint32_t x) { return (uint32_t)s * (uint32_t)ds_sext24(x); };
  // T <- S T while the entries stay < 2^23 (the compiler cannot bound them, and picks v_mul_lo_u32 /
  // v_mad_u64_u32 for about half of such products: the 24-bit forms are spelled out on the device)
  auto mad24 = [](int32_t a, int32_t b, int32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    int32_t d;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
#else
    return (int32_t)((uint32_t)a * (uint32_t)b + (uint32_t)c);
#endif
  };
  auto mul24s = [](int32_t a, int32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    int32_t d;
    asm("v_mul_i32_i24 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
    return d;
#else
    return (int32_t)((uint32_t)a * (uint32_t)b);
#endif
  };
  auto compose24 = [&](const ds_mat& S, const ds_mat& T) {
    return ds_mat{mad24(S.u, T.u, mul24s(S.v, T.q)), mad24(S.u, T.v, mul24s(S.v, T.r)),
                  mad24(S.q, T.u, mul24s(S.r, T.q)), mad24(S.q, T.v, mul24s(S.r, T.r))};
  };
  auto pin = [&](uint32_t off, ds_mat& a, ds_mat& b) { ds_after(off, a.u, a.v, a.q, a.r, b.u, b.v, b.q, b.r); };
  // lookup 0
  uint32_t off = off0;
  uint64_t e = e0;
  fill(0, off);
  ds_mat S = decode(e);
  // lookup 1: F = 2^5 f_1
  uint32_t F = mul32(S.u, f) + mul32(S.v, g), G = mul32(S.q, f) + mul32(S.r, g);
  off = ds_offset<2, -2>(Z, F, G);
  e = load(off);
  fill(1, off);
  ds_mat T = S;
  S = decode(e);
  // lookup 2: F = 2^10 f_2, then the 24-bit window F >> 6
  {
    const uint32_t F2 = mul32(S.u, F) + mul32(S.v, G), G2 = mul32(S.q, F) + mul32(S.r, G);
    off = ds_offset<-3, -7>(Z, F2, G2);
    F = F2 >> 6; G = G2 >> 6;
  }
  e = load(off);
  pin(off, S, T);
  T = compose24(S, T);  // T_2
  fill(2, off);
  S = decode(e);
  // lookups 3-5
  {
    const uint32_t F3 = mul24(S.u, F) + mul24(S.v, G), G3 = mul24(S.q, F) + mul24(S.r, G);
    off = ds_offset<-2, -6>(Z, F3, G3);
    F = F3; G = G3;
  }
  e = load(off);
  pin(off, S, T);
  T = compose24(S, T);  // T_3
  fill(3, off);
  S = decode(e);
  {
    const uint32_t F4 = mul24(S.u, F) + mul24(S.v, G), G4 = mul24(S.q, F) + mul24(S.r, G);
    off = ds_offset<-7, -11>(Z, F4, G4);
    F = F4; G = G4;
  }
  e = load(off);
  pin(off, S, T);
  T = compose24(S, T);  // T_4
  fill(4, off);
  S = decode(e);
  {
    const uint32_t F5 = mul24(S.u, F) + mul24(S.v, G), G5 = mul24(S.q, F) + mul24(S.r, G);
    off = ds_offset<-12, -16>(Z, F5, G5);
  }
  e = load(off);
  pin(off, S, T);
  T = compose24(S, T);  // T_5: entries < 2^25
  fill(5, off);
  S = decode(e);
  t[0] = (int32_t)(mul32(S.u, (uint32_t)T.u) + mul32(S.v, (uint32_t)T.q));
  t[1] = (int32_t)(mul32(S.u, (uint32_t)T.v) + mul32(S.v, (uint32_t)T.r));
  t[2] = (int32_t)(mul32(S.q, (uint32_t)T.u) + mul32(S.r, (uint32_t)T.q));
  t[3] = (int32_t)(mul32(S.q, (uint32_t)T.v) + mul32(S.r, (uint32_t)T.r));
  return Z;
}

// 30 half-delta divsteps by 6 lookups; same return value and t as divsteps30(zeta, f, g, t)
__host__ __device__ __forceinline__ int32_t divsteps30_tab(int32_t zeta, uint32_t f, uint32_t g, int32_t t[4],
                                                           const uint64_t* tab) {
  const int32_t Z = (zeta + DS_TN) * 4096;
  const uint32_t off0 = ds_first(Z, f, g);
  return (divsteps30_tabz(Z, f, g, off0, ds_load(tab, off0), t, tab, [](int, uint32_t) {}) >> 12) - DS_TN;
}

// out = z^-1 (0 -> 0) for a wave-uniform z, table in `tab` (LDS on the device); z as for fe_invert_gcd.
// Half-delta divsteps as fe_invert_gcd, batches of 30 until g = 0 (at most 20: the 590-divstep bound).
__host__ __device__ __forceinline__ void fe_invert_tab(fe& out, const fe& z, const uint64_t* tab) {
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
  int32_t zeta = -1;
  for (int it = 0; it < 20; ++it) {
    int32_t nz = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) nz |= g.v[i];
    if (nz == 0) break;
    int32_t t[4];
    zeta = divsteps30_tab(zeta, (uint32_t)f.v[0], (uint32_t)g.v[0], t, tab);
    inv_update_de(d, e, t);
    inv_update_fg(f, g, t);
  }
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

// ---- wave-uniform inversion with the limb updates spread over lanes --------------------------------
// With table lookups the divsteps are short, and the serial 9-limb updates of f, g, d, e (~200 VALU per batch
// on one wave) become the chain (profiles/r03/finish_stamps_tab.txt).  fe_invert_wave keeps the same
// divsteps (divsteps30_tab on limb 0 of f and g) but holds limb j of every vector in lane j of each 16-lane
// row (the four rows compute the same), so an update is a few lane-parallel instructions plus DPP carries:
//  * f, g (30-bit limbs, exact integers): n_j = (u f + v g)_j >> 30 + lo30((u f + v g)_{j+1}) is the exact
//    division by 2^30 (the limb-0 remainder is 0); a second carry round keeps limbs in [-1, 2^30] (the top
//    limb signed).  Limb 0 stays exact mod 2^30 -- all the divsteps read.
//  * d, e are replaced by the second column (D, E) of the accumulated transition matrix, mod p, in radix
//    2^25.5 with signed limbs: (D, E) <- t (D, E) per batch, two carry rounds (the top carry folds back x19).
//    After k batches f = (A00 p + D x) / 2^30k = +-1, so x^-1 = +-D 2^-30k mod p (DS_INV2K: the constants).
//    No Montgomery correction per batch, no sign tests.
// The same divstep sequence as fe_invert_tab, so the result is the same inverse (it is unique).
static constexpr uint32_t DS_INV2K[21][10] = {  // 2^(-30 k) mod p, k = 0 .. 20, radix 2^25.5 limbs
    {0x0000001u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u, 0x0000000u},
    {0x3fffff4u, 0x1ffffffu, 0x3ffffffu, 0x1ffffffu, 0x3ffffffu, 0x1ffffffu, 0x3ffffffu, 0x1ffffffu, 0x35fffffu, 0x1435e50u},
    {0x3fffff8u, 0x1ffffffu, 0x3ffffffu, 0x1ffffffu, 0x3ffffffu, 0x1ffffffu, 0x3ffffffu, 0x01affffu, 0x39435e5u, 0x0d79435u},
    {0x3ffffeeu, 0x1ffffffu, 0x3ffffffu, 0x1ffffffu, 0x3ffffffu, 0x1ffffffu, 0x0a1afffu, 0x0bca1afu, 0x10d7943u, 0x1e50d79u},
    {0x3fffff4u, 0x1ffffffu, 0x3ffffffu, 0x1ffffffu, 0x3ffffffu, 0x1e50d7fu, 0x06bca1au, 0x1286bcau, 0x35e50d7u, 0x1435e50u},
    {0x3fffff8u, 0x1ffffffu, 0x3ffffffu, 0x1ffffffu, 0x35e50d7u, 0x1435e50u, 0x2f286bcu, 0x01af286u, 0x39435e5u, 0x0d79435u},
    {0x3ffffeeu, 0x1ffffffu, 0x2ffffffu, 0x01af286u, 0x39435e5u, 0x0d79435u, 0x0a1af28u, 0x0bca1afu, 0x10d7943u, 0x1e50d79u},
    {0x3fffff4u, 0x0d7ffffu, 0x0a1af28u, 0x0bca1afu, 0x10d7943u, 0x1e50d79u, 0x06bca1au, 0x1286bcau, 0x35e50d7u, 0x1435e50u},
    {0x10d7ff8u, 0x1e50d79u, 0x06bca1au, 0x1286bcau, 0x35e50d7u, 0x1435e50u, 0x2f286bcu, 0x01af286u, 0x39435e5u, 0x0d79435u},
    {0x35e50d4u, 0x1435e50u, 0x2f286bcu, 0x01af286u, 0x39435e5u, 0x0d79435u, 0x0a1af28u, 0x0bca1afu, 0x10d7943u, 0x0607179u},
    {0x39435d7u, 0x0d79435u, 0x0a1af28u, 0x0bca1afu, 0x10d7943u, 0x1e50d79u, 0x06bca1au, 0x1286bcau, 0x3860717u, 0x17aae72u},
    {0x10d7941u, 0x1e50d79u, 0x06bca1au, 0x1286bcau, 0x35e50d7u, 0x1435e50u, 0x2f286bcu, 0x05c3038u, 0x1b7aae7u, 0x03fd29du},
    {0x35e50ceu, 0x1435e50u, 0x2f286bcu, 0x01af286u, 0x39435e5u, 0x1179435u, 0x0e5c303u, 0x1adbd57u, 0x363fd29u, 0x102209eu},
    {0x39435d3u, 0x0d79435u, 0x0a1af28u, 0x0bca1afu, 0x0717943u, 0x0e72e18u, 0x13adbd5u, 0x1db1fe9u, 0x3502209u, 0x1e6788du},
    {0x10d7938u, 0x1e50d79u, 0x06bca1au, 0x1038bcau, 0x2ae72e1u, 0x129d6deu, 0x13db1feu, 0x1ba8110u, 0x03e6788u, 0x132595au},
    {0x35e50c8u, 0x1435e50u, 0x03038bcu, 0x1d57397u, 0x3d29d6du, 0x009ed8fu, 0x11ba811u, 0x141f33cu, 0x1132595u, 0x1a3cfc7u},
    {0x39435e2u, 0x0e181c5u, 0x1bd5739u, 0x1fe94ebu, 0x2209ed8u, 0x188dd40u, 0x2b41f33u, 0x0e8992cu, 0x31a3cfcu, 0x05242a8u},
    {0x32e181bu, 0x16deab9u, 0x31fe94eu, 0x01104f6u, 0x2788dd4u, 0x195a0f9u, 0x38e8992u, 0x118d1e7u, 0x2c5242au, 0x024e016u},
    {0x1d6dea8u, 0x0d8ff4au, 0x281104fu, 0x133c46eu, 0x2595a0fu, 0x0fc744cu, 0x1518d1eu, 0x0d62921u, 0x3224e01u, 0x06156c6u},
    {0x1ed8ff3u, 0x1d40882u, 0x1f33c46u, 0x192cad0u, 0x3cfc744u, 0x02a8c68u, 0x02d6292u, 0x0d91270u, 0x306156cu, 0x02c905du},
    {0x0dd407eu, 0x00f99e2u, 0x0992cadu, 0x11e7e3au, 0x242a8c6u, 0x0016b14u, 0x18d9127u, 0x1b830abu, 0x022c905u, 0x111a765u},
};

// Lane primitives of the row layout (device: DPP within 16-lane rows; the host harness emulates them).
#if defined(__HIPCC__) && !defined(PBFT_HOST_ONLY)
__device__ __forceinline__ int32_t row_from_below(int32_t x) {  // lane j <- lane j - 1 of its row, lane 0 <- 0
  return __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);  // row_shr:1, bound_ctrl
}
__device__ __forceinline__ int32_t row_from_above(int32_t x) {  // lane j <- lane j + 1 of its row, lane 15 <- 0
  return __builtin_amdgcn_update_dpp(0, x, 0x101, 0xF, 0xF, true);  // row_shl:1, bound_ctrl
}

// Lane j of its row <- lane N of the same 16-lane row (DPP row_newbcast:N).
template <int N>
__device__ __forceinline__ int32_t row_lane(int32_t x) {
  return __builtin_amdgcn_mov_dpp(x, 0x150 + N, 0xF, 0xF, false);  // every lane written: no old value
}

// limb i of v = lane i of this lane's row, i = 0..9
template <int I = 0>
__device__ __forceinline__ void row_limbs(fe& v, int32_t x) {
  if constexpr (I < 10) {
    v.v[I] = (uint32_t)row_lane<I>(x);
    row_limbs<I + 1>(v, x);
  }
}

// out = z^-1 (0 -> 0) for a wave-uniform z (z as for fe_invert_gcd), divstep table `tab` in LDS.  Every lane
// of the wave must call it (the limbs live across lanes); `out` is the same in every lane, carried.
// ROWS: z need only be uniform within each 16-lane row -- the four rows invert their own values (every
// cross-limb read stays inside the row; a row whose g reached 0 early keeps stepping with g = 0, which
// multiplies D by 2^30 per batch as the shared batch count k expects, so its result is unchanged).
template <bool ROWS = false>
__device__ __forceinline__ void fe_invert_wave(fe& out, const fe& z, const uint64_t* tab) {
  static_assert(!ROWS || PBFT_INV_VALU_LOOKUP, "row-wise inversions need the per-row (DPP) lookup operands");
  const int li = (int)(threadIdx.x & 15);  // limb held by this lane
  uint32_t w[8];
  fe_to_words(w, z);
  // f = p, g = z in 30-bit limbs (lanes 0..8; lanes 9..15 hold 0)
  int32_t g = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int b = 30 * i, wi = b >> 5, sh = b & 31;
    uint64_t x = w[wi] >> sh;
    if (wi + 1 < 8) x |= (uint64_t)w[wi + 1] << (32 - sh);
    if (li == i) g = (int32_t)((uint32_t)x & INV_M30);
  }
  int32_t f = li == 0 ? 0x3FFFFFED : li < 8 ? 0x3FFFFFFF : li == 8 ? 0x7FFF : 0;
  // D, E: column (A01, A11) of the accumulated matrix mod p, radix 2^25.5 (lanes 0..9)
  int32_t D = 0, E = li == 0 ? 1 : 0;
  const uint32_t fmask = li < 8 ? INV_M30 : 0xFFFFFFFFu;  // f, g: the top limb (lane 8) keeps its sign
  const int32_t fcarry = li < 8 ? -1 : 0;                  // f, g: carries leave lanes 0..7 only
  const int dsh = (li & 1) ? 25 : 26;
  const uint32_t dmask = (1u << dsh) - 1u;
  const int32_t dlive = li < 10 ? -1 : 0;
  const int32_t w19 = li == 0 ? 19 : 0;  // the carry out of limb 9 re-enters limb 0 times 19
  // (D, E) <- tp (D, E) mod p, two carry rounds (|h| < 2^31, |k| < 2^10 by the limb bounds above; lane 10 picks
  // up limb 9's carry too and the final mask drops it -- that carry re-enters at lane 0, times 19)
  // one of D', E' from its product sum a = x D + y E
  auto de_lane = [&](int64_t a) -> int32_t {
    const int32_t h = (int32_t)(a >> dsh);
    const int32_t h9 = ROWS ? row_lane<9>(h) : __builtin_amdgcn_readlane(h, 9);
    const int64_t n = (int64_t)(int32_t)(((uint32_t)a & dmask) + (uint32_t)row_from_below(h)) + (int64_t)w19 * h9;
    const int32_t kk = (int32_t)(n >> dsh);
    const int32_t k9 = ROWS ? row_lane<9>(kk) : __builtin_amdgcn_readlane(kk, 9);
    return ((int32_t)((uint32_t)n & dmask) + row_from_below(kk) + w19 * k9) & dlive;
  };
  auto update_de = [&](const int32_t tp[4]) {
    const int32_t nD = de_lane((int64_t)tp[0] * D + (int64_t)tp[1] * E);
    const int32_t nE = de_lane((int64_t)tp[2] * D + (int64_t)tp[3] * E);
    D = nD; E = nE;
  };
  int32_t Z = (DS_TN - 1) * 4096;  // zeta = -1, scaled (divsteps30_tabz)
  int32_t tp[4] = {1, 0, 0, 1};  // the previous batch's matrix: (D, E) lag one batch behind f, g
  // the lookups read limb 0 mod 2^30 only: it is exact before the carry round (lane 0 receives no carry), so the
  // next batch's limb 0 reaches the row (row_newbcast:0) and its first entry is read before the carries and the
  // exit test; the test itself reads the limbs before the carries (all zero => g = 0; limbs that cancel only
  // cost one more batch, which leaves the result unchanged, see above)
#if PBFT_INV_VALU_LOOKUP
  auto low = [](int32_t x) { return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x150, 0xF, 0xF, false); };
#else
  auto low = [](int32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane(x); };
#endif
  uint32_t fl = low(f), gl = low(g);
  int32_t gtest = g;
  uint32_t off0 = ds_first(Z, fl, gl);
  uint64_t e0 = ds_load(tab, off0);
  // exit test at the bottom (g = 0: f = +-1): the next batch's first read is issued before the branch (with the
  // test at the top the compiler sinks the read past it)
#if !PBFT_ABL_INV_NOLOOKUP
  auto more = [&](int kk) { return kk < 20 && __ballot(gtest != 0) != 0; };
#else
  auto more = [&](int kk) { return kk < 18; };
#endif
  int k = 0;
  if (more(0)) do {
    int32_t t[4];
    // the previous batch's (D, E) update, independent of this batch's lookups: D' in lookup 0's LDS wait, E' in
    // lookup 1's (divsteps30_tabz pins them after the reads)
    int32_t nD = D, nE = E;
    auto fill = [&](int j, uint32_t off) {
      if (j == 0) {
        ds_after(off, D, E, tp[0], tp[1]);
        nD = de_lane((int64_t)tp[0] * D + (int64_t)tp[1] * E);
      } else if (j == 1) {
        ds_after(off, D, E, tp[2], tp[3]);
        nE = de_lane((int64_t)tp[2] * D + (int64_t)tp[3] * E);
      }
    };
#if PBFT_ABL_INV_NOLOOKUP  // ablation (timing only, results wrong): a fixed matrix instead of the lookups
    t[0] = 1 << 29; t[1] = (int32_t)(fl & 7); t[2] = 3; t[3] = 1 << 28;
    Z -= 30 * 4096;
    fill(0, off0);
    fill(1, off0);
#else
    Z = divsteps30_tabz(Z, fl, gl, off0, e0, t, tab, fill);
#endif
    // f, g <- (t [f, g]) / 2^30: the chain the next lookups wait for
    {
      const int64_t u = t[0], v = t[1], q = t[2], r = t[3];
      const int64_t af = u * f + v * g, ag = q * f + r * g;
      int32_t nf = (int32_t)(af >> 30) + row_from_above((int32_t)((uint32_t)af & INV_M30));
      int32_t ng = (int32_t)(ag >> 30) + row_from_above((int32_t)((uint32_t)ag & INV_M30));
      fl = low(nf); gl = low(ng);
      off0 = ds_first(Z, fl, gl);
      e0 = ds_load(tab, off0);
      gtest = ng;
      f = (int32_t)((uint32_t)nf & fmask) + row_from_below((nf >> 30) & fcarry);
      g = (int32_t)((uint32_t)ng & fmask) + row_from_below((ng >> 30) & fcarry);
    }
    D = nD; E = nE;
    tp[0] = t[0]; tp[1] = t[1]; tp[2] = t[2]; tp[3] = t[3];
  } while (more(++k));
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" ::"v"(e0));  // the last speculative read is live on the exit edge too: it stays ahead of the branch
#endif
  update_de(tp);
  // x^-1 = +-D 2^(-30 k): f = +1 iff its limb 0 is 1
  const bool neg = ((uint32_t)(ROWS ? row_lane<0>(f) : __builtin_amdgcn_readfirstlane(f)) & INV_M30) != 1u;
  fe d, c, p2;
  if constexpr (ROWS) row_limbs(p2, D);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    if constexpr (!ROWS) p2.v[i] = (uint32_t)__builtin_amdgcn_readlane(D, i);
    // limbs in [-2^12, 2^26 + 2^12]: + 2p makes them positive and within fe_mul's operand bounds
    d.v[i] = p2.v[i] + (i == 0 ? 0x7FFFFDAu : (i & 1) ? 0x3FFFFFEu : 0x7FFFFFEu);
    c.v[i] = DS_INV2K[k][i];
  }
  fe_mul(out, d, c);
  if (neg) { fe_neg(p2, out); fe_carry(p2); out = p2; }
}
#endif

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
