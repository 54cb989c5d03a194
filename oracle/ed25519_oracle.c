/*
 * TEST INFRASTRUCTURE — NOT PRODUCT CODE.
 *
 * Plain-C CPU restatement of Ed25519 verify_strict / RFC 8032 sign, used only
 * by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg (as the
 * checker and as the "port" CPU baseline).  It shares no code with the HIP
 * product path: radix 2^51 limbs with unsigned __int128 products here, radix
 * 2^25.5 on the GPU.
 *
 * Semantics restated (the reference's crypto lives in un-vendored crates, see
 * oracle/ed25519_ref.py for the full citation list):
 *   ed25519-dalek 1.0.1 PublicKey::verify_strict    (Cargo.lock:668-679)
 *   curve25519-dalek 3.2.1 decompress / is_small_order / from_hash
 *                                                    (Cargo.lock:604-614)
 *   sha2 0.9.9 SHA-512                               (Cargo.lock:2784-2787)
 * Call sites it slots into: validate_prepare src/behavior.rs:159-175 and
 * validate_commit src/behavior.rs:184-195 (signature checks are TODOs at
 * src/behavior.rs:127 and :185).
 *
 * Pinned against: RFC 8032 §7.1 KATs, the pure-Python restatement
 * (oracle/ed25519_ref.py) on every golden vector class, and libsodium/OpenSSL
 * on the classes where their semantics coincide (tests/test_oracle.py).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <pthread.h>
#include <stdlib.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[5]; } fe;
#define M51 ((1ULL << 51) - 1)

/* ---------------- field GF(2^255-19), radix 2^51 ---------------- */
static void fe_frombytes(fe *h, const uint8_t s[32]) {
  /* curve25519-dalek FieldElement::from_bytes: bit 255 ignored, no < p check */
  uint64_t w[4];
  for (int i = 0; i < 4; ++i) {
    w[i] = 0;
    for (int j = 0; j < 8; ++j) w[i] |= (uint64_t)s[8 * i + j] << (8 * j);
  }
  h->v[0] = w[0] & M51;
  h->v[1] = ((w[0] >> 51) | (w[1] << 13)) & M51;
  h->v[2] = ((w[1] >> 38) | (w[2] << 26)) & M51;
  h->v[3] = ((w[2] >> 25) | (w[3] << 39)) & M51;
  h->v[4] = (w[3] >> 12) & M51;
}
static void fe_carry(fe *h) {
  uint64_t c;
  for (int k = 0; k < 2; ++k) {
    c = h->v[0] >> 51; h->v[0] &= M51; h->v[1] += c;
    c = h->v[1] >> 51; h->v[1] &= M51; h->v[2] += c;
    c = h->v[2] >> 51; h->v[2] &= M51; h->v[3] += c;
    c = h->v[3] >> 51; h->v[3] &= M51; h->v[4] += c;
    c = h->v[4] >> 51; h->v[4] &= M51; h->v[0] += 19 * c;
  }
}
static void fe_tobytes(uint8_t s[32], const fe *f) {
  fe t = *f;
  fe_carry(&t);
  /* now t < 2^255 + small; subtract p if t >= p */
  uint64_t q = (t.v[0] + 19) >> 51;
  q = (t.v[1] + q) >> 51;
  q = (t.v[2] + q) >> 51;
  q = (t.v[3] + q) >> 51;
  q = (t.v[4] + q) >> 51;
  t.v[0] += 19 * q;
  uint64_t c;
  c = t.v[0] >> 51; t.v[0] &= M51; t.v[1] += c;
  c = t.v[1] >> 51; t.v[1] &= M51; t.v[2] += c;
  c = t.v[2] >> 51; t.v[2] &= M51; t.v[3] += c;
  c = t.v[3] >> 51; t.v[3] &= M51; t.v[4] += c;
  t.v[4] &= M51;
  uint64_t w[4];
  w[0] = t.v[0] | (t.v[1] << 51);
  w[1] = (t.v[1] >> 13) | (t.v[2] << 38);
  w[2] = (t.v[2] >> 26) | (t.v[3] << 25);
  w[3] = (t.v[3] >> 39) | (t.v[4] << 12);
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}
static void fe_0(fe *h) { memset(h, 0, sizeof *h); }
static void fe_1(fe *h) { fe_0(h); h->v[0] = 1; }
static void fe_add(fe *h, const fe *f, const fe *g) {
  for (int i = 0; i < 5; ++i) h->v[i] = f->v[i] + g->v[i];
  fe_carry(h);
}
static void fe_sub(fe *h, const fe *f, const fe *g) {
  /* add 4p before subtracting (limbs of g are < 2^52 after carry) */
  static const uint64_t p4[5] = {0x1FFFFFFFFFFFB4ULL, 0x1FFFFFFFFFFFFCULL, 0x1FFFFFFFFFFFFCULL,
                                 0x1FFFFFFFFFFFFCULL, 0x1FFFFFFFFFFFFCULL};
  for (int i = 0; i < 5; ++i) h->v[i] = f->v[i] + p4[i] - g->v[i];
  fe_carry(h);
}
static void fe_neg(fe *h, const fe *f) { fe z; fe_0(&z); fe_sub(h, &z, f); }
static void fe_mul(fe *h, const fe *f, const fe *g) {
  const uint64_t *a = f->v, *b = g->v;
  uint64_t b19[5];
  for (int i = 0; i < 5; ++i) b19[i] = 19 * b[i];
  u128 r0 = (u128)a[0] * b[0] + (u128)a[1] * b19[4] + (u128)a[2] * b19[3] + (u128)a[3] * b19[2] + (u128)a[4] * b19[1];
  u128 r1 = (u128)a[0] * b[1] + (u128)a[1] * b[0] + (u128)a[2] * b19[4] + (u128)a[3] * b19[3] + (u128)a[4] * b19[2];
  u128 r2 = (u128)a[0] * b[2] + (u128)a[1] * b[1] + (u128)a[2] * b[0] + (u128)a[3] * b19[4] + (u128)a[4] * b19[3];
  u128 r3 = (u128)a[0] * b[3] + (u128)a[1] * b[2] + (u128)a[2] * b[1] + (u128)a[3] * b[0] + (u128)a[4] * b19[4];
  u128 r4 = (u128)a[0] * b[4] + (u128)a[1] * b[3] + (u128)a[2] * b[2] + (u128)a[3] * b[1] + (u128)a[4] * b[0];
  uint64_t c;
  r1 += (uint64_t)(r0 >> 51); uint64_t h0 = (uint64_t)r0 & M51;
  r2 += (uint64_t)(r1 >> 51); uint64_t h1 = (uint64_t)r1 & M51;
  r3 += (uint64_t)(r2 >> 51); uint64_t h2 = (uint64_t)r2 & M51;
  r4 += (uint64_t)(r3 >> 51); uint64_t h3 = (uint64_t)r3 & M51;
  c = (uint64_t)(r4 >> 51); uint64_t h4 = (uint64_t)r4 & M51;
  h0 += 19 * c;
  c = h0 >> 51; h0 &= M51; h1 += c;
  h->v[0] = h0; h->v[1] = h1; h->v[2] = h2; h->v[3] = h3; h->v[4] = h4;
}
static void fe_sq(fe *h, const fe *f) { fe_mul(h, f, f); }
static void fe_sqn(fe *h, const fe *f, int n) { *h = *f; for (int i = 0; i < n; ++i) fe_sq(h, h); }
/* z^(2^250 - 1), shared by invert and pow22523 */
static void fe_pow250(fe *out, fe *z11, const fe *z) {
  fe t0, t1, z2, z9, z2_5_0, z2_10_0, z2_20_0, z2_50_0, z2_100_0;
  fe_sq(&z2, z);
  fe_sqn(&t0, &z2, 2);
  fe_mul(&z9, &t0, z);
  fe_mul(z11, &z9, &z2);
  fe_sq(&t0, z11);
  fe_mul(&z2_5_0, &t0, &z9);
  fe_sqn(&t0, &z2_5_0, 5); fe_mul(&z2_10_0, &t0, &z2_5_0);
  fe_sqn(&t0, &z2_10_0, 10); fe_mul(&z2_20_0, &t0, &z2_10_0);
  fe_sqn(&t0, &z2_20_0, 20); fe_mul(&t1, &t0, &z2_20_0);
  fe_sqn(&t0, &t1, 10); fe_mul(&z2_50_0, &t0, &z2_10_0);
  fe_sqn(&t0, &z2_50_0, 50); fe_mul(&z2_100_0, &t0, &z2_50_0);
  fe_sqn(&t0, &z2_100_0, 100); fe_mul(&t1, &t0, &z2_100_0);
  fe_sqn(&t0, &t1, 50); fe_mul(out, &t0, &z2_50_0);
}
static void fe_invert(fe *out, const fe *z) {
  fe t, z11;
  fe_pow250(&t, &z11, z);
  fe_sqn(&t, &t, 5);
  fe_mul(out, &t, &z11); /* z^(2^255 - 21) */
}
static void fe_pow22523(fe *out, const fe *z) {
  fe t, z11;
  fe_pow250(&t, &z11, z);
  fe_sqn(&t, &t, 2);
  fe_mul(out, &t, z); /* z^(2^252 - 3) */
}
static int fe_eq(const fe *a, const fe *b) {
  uint8_t x[32], y[32];
  fe_tobytes(x, a); fe_tobytes(y, b);
  return memcmp(x, y, 32) == 0;
}
static int fe_iszero(const fe *a) { fe z; fe_0(&z); return fe_eq(a, &z); }
static int fe_isneg(const fe *a) { uint8_t x[32]; fe_tobytes(x, a); return x[0] & 1; }

static fe FE_D, FE_D2, FE_SQRTM1;
static const uint8_t D_BYTES[32] = {
  0xa3,0x78,0x59,0x13,0xca,0x4d,0xeb,0x75,0xab,0xd8,0x41,0x41,0x4d,0x0a,0x70,0x00,
  0x98,0xe8,0x79,0x77,0x79,0x40,0xc7,0x8c,0x73,0xfe,0x6f,0x2b,0xee,0x6c,0x03,0x52};
static const uint8_t SQRTM1_BYTES[32] = {
  0xb0,0xa0,0x0e,0x4a,0x27,0x1b,0xee,0xc4,0x78,0xe4,0x2f,0xad,0x06,0x18,0x43,0x2f,
  0xa7,0xd7,0xfb,0x3d,0x99,0x00,0x4d,0x2b,0x0b,0xdf,0xc1,0x4f,0x80,0x24,0x83,0x2b};
static const uint8_t BY_BYTES[32] = {
  0x58,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,
  0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66,0x66};

/* ---------------- group: extended twisted Edwards (a = -1) ---------------- */
typedef struct { fe X, Y, Z, T; } ge;

static void ge_ident(ge *p) { fe_0(&p->X); fe_1(&p->Y); fe_1(&p->Z); fe_0(&p->T); }
static void ge_add(ge *r, const ge *p, const ge *q) {
  fe a, b, c, d, e, f, g, h, t;
  fe_sub(&a, &p->Y, &p->X); fe_sub(&t, &q->Y, &q->X); fe_mul(&a, &a, &t);
  fe_add(&b, &p->Y, &p->X); fe_add(&t, &q->Y, &q->X); fe_mul(&b, &b, &t);
  fe_mul(&c, &p->T, &q->T); fe_mul(&c, &c, &FE_D2);
  fe_mul(&d, &p->Z, &q->Z); fe_add(&d, &d, &d);
  fe_sub(&e, &b, &a); fe_sub(&f, &d, &c); fe_add(&g, &d, &c); fe_add(&h, &b, &a);
  fe_mul(&r->X, &e, &f); fe_mul(&r->Y, &g, &h); fe_mul(&r->Z, &f, &g); fe_mul(&r->T, &e, &h);
}
static void ge_dbl(ge *r, const ge *p) {
  /* dbl-2008-hwcd for a = -1 */
  fe a, b, c, e, g, f, h, t;
  fe_sq(&a, &p->X); fe_sq(&b, &p->Y); fe_sq(&c, &p->Z); fe_add(&c, &c, &c);
  fe_add(&t, &p->X, &p->Y); fe_sq(&t, &t);
  fe_add(&h, &a, &b);            /* H = A + B */
  fe_sub(&e, &h, &t);            /* E = H - (X+Y)^2  (= -(2XY)) */
  fe_sub(&g, &a, &b);            /* G = A - B  (= aA + B with a=-1, negated) */
  fe_add(&f, &c, &g);            /* F = C + G */
  fe_mul(&r->X, &e, &f); fe_mul(&r->Y, &g, &h); fe_mul(&r->T, &e, &h); fe_mul(&r->Z, &f, &g);
}
static void ge_neg(ge *r, const ge *p) { *r = *p; fe_neg(&r->X, &p->X); fe_neg(&r->T, &p->T); }
static int ge_eq(const ge *p, const ge *q) {
  fe a, b;
  fe_mul(&a, &p->X, &q->Z); fe_mul(&b, &q->X, &p->Z);
  if (!fe_eq(&a, &b)) return 0;
  fe_mul(&a, &p->Y, &q->Z); fe_mul(&b, &q->Y, &p->Z);
  return fe_eq(&a, &b);
}
static int ge_is_small_order(const ge *p) {
  ge q; ge_dbl(&q, p); ge_dbl(&q, &q); ge_dbl(&q, &q);
  ge id; ge_ident(&id);
  return ge_eq(&q, &id);
}
/* CompressedEdwardsY::decompress (curve25519-dalek 3.2.1) */
static int ge_decompress(ge *p, const uint8_t s[32]) {
  fe y, yy, u, v, v3, v7, r, chk, one, nu, nui;
  fe_frombytes(&y, s);
  fe_1(&one);
  fe_sq(&yy, &y);
  fe_sub(&u, &yy, &one);
  fe_mul(&v, &yy, &FE_D); fe_add(&v, &v, &one);
  /* sqrt_ratio_i(u, v) */
  fe_sq(&v3, &v); fe_mul(&v3, &v3, &v);
  fe_sq(&v7, &v3); fe_mul(&v7, &v7, &v);
  fe_mul(&r, &u, &v7); fe_pow22523(&r, &r); fe_mul(&r, &r, &u); fe_mul(&r, &r, &v3);
  fe_sq(&chk, &r); fe_mul(&chk, &chk, &v);
  fe_neg(&nu, &u); fe_mul(&nui, &nu, &FE_SQRTM1);
  int correct = fe_eq(&chk, &u), flipped = fe_eq(&chk, &nu), flipped_i = fe_eq(&chk, &nui);
  if (flipped || flipped_i) fe_mul(&r, &r, &FE_SQRTM1);
  if (fe_isneg(&r)) fe_neg(&r, &r);
  if (!(correct || flipped)) return 0;
  if (s[31] >> 7) fe_neg(&r, &r);
  p->X = r; p->Y = y; fe_1(&p->Z); fe_mul(&p->T, &r, &y);
  return 1;
}
static void ge_compress(uint8_t s[32], const ge *p) {
  fe zi, x, y;
  fe_invert(&zi, &p->Z);
  fe_mul(&x, &p->X, &zi); fe_mul(&y, &p->Y, &zi);
  fe_tobytes(s, &y);
  s[31] |= (uint8_t)(fe_isneg(&x) << 7);
}

/* [a]P + [b]Q, 4-bit fixed windows (interleaved); a, b little-endian 32 bytes */
static void ge_double_scalarmult(ge *r, const uint8_t a[32], const ge *P, const uint8_t b[32], const ge *Q) {
  ge tp[16], tq[16];
  ge_ident(&tp[0]); ge_ident(&tq[0]);
  tp[1] = *P; tq[1] = *Q;
  for (int i = 2; i < 16; ++i) { ge_add(&tp[i], &tp[i - 1], P); ge_add(&tq[i], &tq[i - 1], Q); }
  ge acc; ge_ident(&acc);
  for (int i = 63; i >= 0; --i) {
    ge_dbl(&acc, &acc); ge_dbl(&acc, &acc); ge_dbl(&acc, &acc); ge_dbl(&acc, &acc);
    int da = (a[i >> 1] >> ((i & 1) * 4)) & 15, db = (b[i >> 1] >> ((i & 1) * 4)) & 15;
    if (da) ge_add(&acc, &acc, &tp[da]);
    if (db) ge_add(&acc, &acc, &tq[db]);
  }
  *r = acc;
}

static ge GE_B;
static pthread_once_t init_once = PTHREAD_ONCE_INIT;
static void init_consts(void) {
  fe_frombytes(&FE_D, D_BYTES);
  fe_add(&FE_D2, &FE_D, &FE_D);
  fe_frombytes(&FE_SQRTM1, SQRTM1_BYTES);
  ge_decompress(&GE_B, BY_BYTES);
}

/* ---------------- scalars mod L ---------------- */
static const uint8_t L_BYTES[32] = {
  0xed,0xd3,0xf5,0x5c,0x1a,0x63,0x12,0x58,0xd6,0x9c,0xf7,0xa2,0xde,0xf9,0xde,0x14,
  0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0x10};
static int sc_lt_L(const uint8_t s[32]) {
  for (int i = 31; i >= 0; --i) {
    if (s[i] < L_BYTES[i]) return 1;
    if (s[i] > L_BYTES[i]) return 0;
  }
  return 0;
}
/* x (n bytes, little-endian) mod L by shift-and-subtract, bit at a time */
static void sc_reduce(uint8_t out[32], const uint8_t *x, int n) {
  uint64_t r[5] = {0, 0, 0, 0, 0}, l[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < 32; ++i) l[i / 8] |= (uint64_t)L_BYTES[i] << (8 * (i % 8));
  for (int bit = 8 * n - 1; bit >= 0; --bit) {
    uint64_t in = (x[bit >> 3] >> (bit & 7)) & 1;
    for (int i = 4; i > 0; --i) r[i] = (r[i] << 1) | (r[i - 1] >> 63);
    r[0] = (r[0] << 1) | in;
    /* if r >= L: r -= L */
    int ge_ = 1;
    for (int i = 4; i >= 0; --i) {
      if (r[i] > l[i]) { ge_ = 1; break; }
      if (r[i] < l[i]) { ge_ = 0; break; }
    }
    if (ge_) {
      uint64_t bo = 0;
      for (int i = 0; i < 5; ++i) {
        u128 d = (u128)r[i] - l[i] - bo;
        r[i] = (uint64_t)d;
        bo = (uint64_t)(d >> 64) & 1;
      }
    }
  }
  for (int i = 0; i < 32; ++i) out[i] = (uint8_t)(r[i / 8] >> (8 * (i % 8)));
}
/* (a*b + c) mod L */
static void sc_muladd(uint8_t out[32], const uint8_t a[32], const uint8_t b[32], const uint8_t c[32]) {
  uint32_t prod[17] = {0};
  uint64_t t[16] = {0};
  uint32_t aw[8], bw[8];
  for (int i = 0; i < 8; ++i) {
    aw[i] = a[4 * i] | (a[4 * i + 1] << 8) | (a[4 * i + 2] << 16) | ((uint32_t)a[4 * i + 3] << 24);
    bw[i] = b[4 * i] | (b[4 * i + 1] << 8) | (b[4 * i + 2] << 16) | ((uint32_t)b[4 * i + 3] << 24);
  }
  u128 acc = 0;
  for (int k = 0; k < 16; ++k) {
    for (int i = 0; i < 8; ++i) {
      int j = k - i;
      if (j >= 0 && j < 8) acc += (uint64_t)aw[i] * bw[j];
    }
    if (k < 8) acc += (uint32_t)(c[4 * k] | (c[4 * k + 1] << 8) | (c[4 * k + 2] << 16) | ((uint32_t)c[4 * k + 3] << 24));
    t[k] = (uint32_t)acc;
    acc >>= 32;
  }
  for (int k = 0; k < 16; ++k) prod[k] = (uint32_t)t[k];
  uint8_t bytes[64];
  for (int k = 0; k < 16; ++k)
    for (int j = 0; j < 4; ++j) bytes[4 * k + j] = (uint8_t)(prod[k] >> (8 * j));
  sc_reduce(out, bytes, 64);
}

/* ---------------- SHA-512 (FIPS 180-4) ---------------- */
static const uint64_t K512[80] = {
  0x428a2f98d728ae22ULL,0x7137449123ef65cdULL,0xb5c0fbcfec4d3b2fULL,0xe9b5dba58189dbbcULL,0x3956c25bf348b538ULL,
  0x59f111f1b605d019ULL,0x923f82a4af194f9bULL,0xab1c5ed5da6d8118ULL,0xd807aa98a3030242ULL,0x12835b0145706fbeULL,
  0x243185be4ee4b28cULL,0x550c7dc3d5ffb4e2ULL,0x72be5d74f27b896fULL,0x80deb1fe3b1696b1ULL,0x9bdc06a725c71235ULL,
  0xc19bf174cf692694ULL,0xe49b69c19ef14ad2ULL,0xefbe4786384f25e3ULL,0x0fc19dc68b8cd5b5ULL,0x240ca1cc77ac9c65ULL,
  0x2de92c6f592b0275ULL,0x4a7484aa6ea6e483ULL,0x5cb0a9dcbd41fbd4ULL,0x76f988da831153b5ULL,0x983e5152ee66dfabULL,
  0xa831c66d2db43210ULL,0xb00327c898fb213fULL,0xbf597fc7beef0ee4ULL,0xc6e00bf33da88fc2ULL,0xd5a79147930aa725ULL,
  0x06ca6351e003826fULL,0x142929670a0e6e70ULL,0x27b70a8546d22ffcULL,0x2e1b21385c26c926ULL,0x4d2c6dfc5ac42aedULL,
  0x53380d139d95b3dfULL,0x650a73548baf63deULL,0x766a0abb3c77b2a8ULL,0x81c2c92e47edaee6ULL,0x92722c851482353bULL,
  0xa2bfe8a14cf10364ULL,0xa81a664bbc423001ULL,0xc24b8b70d0f89791ULL,0xc76c51a30654be30ULL,0xd192e819d6ef5218ULL,
  0xd69906245565a910ULL,0xf40e35855771202aULL,0x106aa07032bbd1b8ULL,0x19a4c116b8d2d0c8ULL,0x1e376c085141ab53ULL,
  0x2748774cdf8eeb99ULL,0x34b0bcb5e19b48a8ULL,0x391c0cb3c5c95a63ULL,0x4ed8aa4ae3418acbULL,0x5b9cca4f7763e373ULL,
  0x682e6ff3d6b2b8a3ULL,0x748f82ee5defb2fcULL,0x78a5636f43172f60ULL,0x84c87814a1f0ab72ULL,0x8cc702081a6439ecULL,
  0x90befffa23631e28ULL,0xa4506cebde82bde9ULL,0xbef9a3f7b2c67915ULL,0xc67178f2e372532bULL,0xca273eceea26619cULL,
  0xd186b8c721c0c207ULL,0xeada7dd6cde0eb1eULL,0xf57d4f7fee6ed178ULL,0x06f067aa72176fbaULL,0x0a637dc5a2c898a6ULL,
  0x113f9804bef90daeULL,0x1b710b35131c471bULL,0x28db77f523047d84ULL,0x32caab7b40c72493ULL,0x3c9ebe0a15c9bebcULL,
  0x431d67c49c100d4cULL,0x4cc5d4becb3e42b6ULL,0x597f299cfc657e2aULL,0x5fcb6fab3ad6faecULL,0x6c44198c4a475817ULL};
#define ROR64(x, n) (((x) >> (n)) | ((x) << (64 - (n))))
static void sha512_block(uint64_t H[8], const uint8_t blk[128]) {
  uint64_t W[80];
  for (int t = 0; t < 16; ++t) {
    W[t] = 0;
    for (int j = 0; j < 8; ++j) W[t] = (W[t] << 8) | blk[8 * t + j];
  }
  for (int t = 16; t < 80; ++t) {
    uint64_t s0 = ROR64(W[t - 15], 1) ^ ROR64(W[t - 15], 8) ^ (W[t - 15] >> 7);
    uint64_t s1 = ROR64(W[t - 2], 19) ^ ROR64(W[t - 2], 61) ^ (W[t - 2] >> 6);
    W[t] = W[t - 16] + s0 + W[t - 7] + s1;
  }
  uint64_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
  for (int t = 0; t < 80; ++t) {
    uint64_t S1 = ROR64(e, 14) ^ ROR64(e, 18) ^ ROR64(e, 41);
    uint64_t ch = (e & f) ^ (~e & g);
    uint64_t T1 = h + S1 + ch + K512[t] + W[t];
    uint64_t S0 = ROR64(a, 28) ^ ROR64(a, 34) ^ ROR64(a, 39);
    uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint64_t T2 = S0 + mj;
    h = g; g = f; f = e; e = d + T1; d = c; c = b; b = a; a = T1 + T2;
  }
  H[0] += a; H[1] += b; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
}
/* SHA-512 over the concatenation of up to three segments */
static void sha512_3(uint8_t out[64], const uint8_t *p1, size_t n1, const uint8_t *p2, size_t n2,
                     const uint8_t *p3, size_t n3) {
  uint64_t H[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                   0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  uint8_t blk[128];
  size_t fill = 0, total = n1 + n2 + n3;
  const uint8_t *segs[3] = {p1, p2, p3};
  size_t lens[3] = {n1, n2, n3};
  for (int s = 0; s < 3; ++s) {
    for (size_t i = 0; i < lens[s]; ++i) {
      blk[fill++] = segs[s][i];
      if (fill == 128) { sha512_block(H, blk); fill = 0; }
    }
  }
  blk[fill++] = 0x80;
  if (fill > 112) { memset(blk + fill, 0, 128 - fill); sha512_block(H, blk); fill = 0; }
  memset(blk + fill, 0, 128 - fill);
  uint64_t bits = (uint64_t)total * 8;
  for (int j = 0; j < 8; ++j) blk[127 - j] = (uint8_t)(bits >> (8 * j));
  sha512_block(H, blk);
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) out[8 * i + j] = (uint8_t)(H[i] >> (56 - 8 * j));
}

/* ---------------- public oracle API ---------------- */
void oracle_sha512(uint8_t out[64], const uint8_t *m, size_t n) { sha512_3(out, m, n, NULL, 0, NULL, 0); }

int oracle_key_ok(const uint8_t pk[32]) {
  pthread_once(&init_once, init_consts);
  ge A;
  if (!ge_decompress(&A, pk)) return 0;
  return !ge_is_small_order(&A);
}

/* verify_strict given the key already decoded the way a dalek PublicKey holds it: negA = -A (a_ok = 0: the
 * encoding did not decompress or A has small order -- every signature under it is rejected) */
static int verify_strict_negA(const ge *negA, int a_ok, const uint8_t pk[32], const uint8_t sig[64],
                              const uint8_t *msg, size_t len) {
  const uint8_t *s = sig + 32;
  if (!sc_lt_L(s)) return 0;                       /* check_scalar */
  if (!a_ok) return 0;
  ge R, Rp;
  if (!ge_decompress(&R, sig)) return 0;           /* signature.R.decompress() */
  if (ge_is_small_order(&R)) return 0;
  uint8_t h[64], k[32];
  sha512_3(h, sig, 32, pk, 32, msg, len);          /* R || A || M, raw bytes */
  sc_reduce(k, h, 64);                             /* Scalar::from_hash */
  ge_double_scalarmult(&Rp, k, negA, s, &GE_B);   /* [k](-A) + [s]B */
  return ge_eq(&Rp, &R);                           /* EdwardsPoint == */
}

/* PublicKey::from_bytes (decompression) + the small-order rejection verify_strict applies to A */
static int decode_key(ge *negA, const uint8_t pk[32]) {
  ge A;
  if (!ge_decompress(&A, pk)) return 0;
  if (ge_is_small_order(&A)) return 0;
  ge_neg(negA, &A);
  return 1;
}

/* ed25519-dalek 1.0.1 verify_strict: 1 = accept, 0 = reject */
int oracle_verify_strict(const uint8_t pk[32], const uint8_t sig[64], const uint8_t *msg, size_t len) {
  pthread_once(&init_once, init_consts);
  if (!sc_lt_L(sig + 32)) return 0;                /* check_scalar first, as dalek */
  ge negA;
  const int a_ok = decode_key(&negA, pk);
  return verify_strict_negA(&negA, a_ok, pk, sig, msg, len);
}

void oracle_public_key(uint8_t pk[32], const uint8_t seed[32]) {
  pthread_once(&init_once, init_consts);
  uint8_t h[64];
  oracle_sha512(h, seed, 32);
  h[0] &= 248; h[31] &= 127; h[31] |= 64;
  ge P, id; ge_ident(&id);
  uint8_t zero[32] = {0};
  ge_double_scalarmult(&P, h, &GE_B, zero, &id);
  ge_compress(pk, &P);
}

/* RFC 8032 deterministic signature */
void oracle_sign(uint8_t sig[64], const uint8_t seed[32], const uint8_t *msg, size_t len) {
  pthread_once(&init_once, init_consts);
  uint8_t h[64], pk[32], rh[64], r[32], kh[64], k[32];
  oracle_sha512(h, seed, 32);
  h[0] &= 248; h[31] &= 127; h[31] |= 64;
  ge P, id; ge_ident(&id);
  uint8_t zero[32] = {0};
  ge_double_scalarmult(&P, h, &GE_B, zero, &id);
  ge_compress(pk, &P);
  sha512_3(rh, h + 32, 32, msg, len, NULL, 0);
  sc_reduce(r, rh, 64);
  ge_double_scalarmult(&P, r, &GE_B, zero, &id);
  ge_compress(sig, &P);
  sha512_3(kh, sig, 32, pk, 32, msg, len);
  sc_reduce(k, kh, 64);
  uint8_t a[32];
  memcpy(a, h, 32);
  sc_muladd(sig + 32, k, a, r);
}

/* Batch verify over the same SoA contract as include/pbft_verify.h:
 * R[N*32], S[N*32], key_idx[N], msg[N*msg_stride] (msg_len bytes used),
 * keys[n_keys*32].  bitmap_out[ceil(N/64)] LSB-first; bits past N zero. */
typedef struct {
  const uint8_t *R, *S, *msg, *keys; const uint16_t *key_idx;
  uint32_t msg_len, msg_stride, n_keys; uint64_t lo, hi; uint8_t *acc;
  const ge *negA; const uint8_t *a_ok;
} job_t;
static void *batch_worker(void *arg) {
  job_t *j = (job_t *)arg;
  uint8_t sig[64];
  for (uint64_t i = j->lo; i < j->hi; ++i) {
    uint16_t ki = j->key_idx[i];
    if (ki >= j->n_keys) { j->acc[i] = 0; continue; }
    memcpy(sig, j->R + 32 * i, 32);
    memcpy(sig + 32, j->S + 32 * i, 32);
    j->acc[i] = (uint8_t)verify_strict_negA(&j->negA[ki], j->a_ok[ki], j->keys + 32 * (size_t)ki, sig,
                                            j->msg + (size_t)j->msg_stride * i, j->msg_len);
  }
  return NULL;
}
/* Like a libp2p replica, which decodes each peer's key once (PublicKey::from_bytes) and verifies many
 * signatures under it, the batch decodes the n_keys keys first (-A and the small-order check), then
 * verifies every signature against the decoded key. */
int oracle_verify_batch(const uint8_t *keys, uint32_t n_keys, const uint8_t *R, const uint8_t *S,
                        const uint16_t *key_idx, const uint8_t *msg, uint32_t msg_len, uint32_t msg_stride,
                        uint64_t N, uint8_t *accept_bytes, int nthreads) {
  pthread_once(&init_once, init_consts);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  ge *negA = (ge *)malloc(sizeof(ge) * (n_keys ? n_keys : 1));
  uint8_t *a_ok = (uint8_t *)malloc(n_keys ? n_keys : 1);
  if (!negA || !a_ok) { free(negA); free(a_ok); return -1; }
  for (uint32_t k = 0; k < n_keys; ++k) a_ok[k] = (uint8_t)decode_key(&negA[k], keys + 32 * (size_t)k);
  pthread_t th[256];
  job_t jobs[256];
  uint64_t per = (N + nthreads - 1) / nthreads;
  int started = 0, rc = 0;
  for (int t = 0; t < nthreads; ++t) {
    uint64_t lo = per * t, hi = lo + per > N ? N : lo + per;
    if (lo >= hi) break;
    jobs[t] = (job_t){R, S, msg, keys, key_idx, msg_len, msg_stride, n_keys, lo, hi, accept_bytes, negA, a_ok};
    if (pthread_create(&th[t], NULL, batch_worker, &jobs[t]) != 0) { rc = -1; break; }
    ++started;
  }
  for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
  free(negA);
  free(a_ok);
  return rc;
}

typedef struct {
  const uint8_t *seeds; const uint16_t *key_idx; const uint8_t *msg; uint32_t msg_len, msg_stride;
  uint64_t lo, hi; uint8_t *R, *S;
} sjob_t;
static void *sign_worker(void *arg) {
  sjob_t *j = (sjob_t *)arg;
  uint8_t sig[64];
  for (uint64_t i = j->lo; i < j->hi; ++i) {
    oracle_sign(sig, j->seeds + 32 * (size_t)j->key_idx[i], j->msg + (size_t)j->msg_stride * i, j->msg_len);
    memcpy(j->R + 32 * i, sig, 32);
    memcpy(j->S + 32 * i, sig + 32, 32);
  }
  return NULL;
}
int oracle_sign_batch(const uint8_t *seeds, const uint16_t *key_idx, const uint8_t *msg, uint32_t msg_len,
                      uint32_t msg_stride, uint64_t N, uint8_t *R, uint8_t *S, int nthreads) {
  pthread_once(&init_once, init_consts);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  sjob_t jobs[256];
  uint64_t per = (N + nthreads - 1) / nthreads;
  int started = 0;
  for (int t = 0; t < nthreads; ++t) {
    uint64_t lo = per * t, hi = lo + per > N ? N : lo + per;
    if (lo >= hi) break;
    jobs[t] = (sjob_t){seeds, key_idx, msg, msg_len, msg_stride, lo, hi, R, S};
    if (pthread_create(&th[t], NULL, sign_worker, &jobs[t]) != 0) return -1;
    ++started;
  }
  for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
  return 0;
}
