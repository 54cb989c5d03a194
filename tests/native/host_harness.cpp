// TEST INFRASTRUCTURE: the product's __host__ __device__ arithmetic
// (pbft_amd/csrc/*.h) compiled for the HOST, so tests/test_host_harness.py can
// check fields, hashing, scalar reduction, comb tables and the full per-lane
// verify against the oracle in a container without a GPU.  Never loaded by the
// product path (pbft_amd/ loads only libpbft_verify.so, which needs a GPU).
#include "../../pbft_amd/csrc/inv25519.h"
#include "../../pbft_amd/csrc/verify_core.h"
#include <sys/mman.h>
#include <unistd.h>

#include <cstring>
#include <vector>

using namespace pbft;

static void words_from_bytes(uint32_t w[8], const uint8_t* b) {
  for (int i = 0; i < 8; ++i) w[i] = b[4 * i] | (b[4 * i + 1] << 8) | (b[4 * i + 2] << 16) | ((uint32_t)b[4 * i + 3] << 24);
}
static void bytes_from_words(uint8_t* b, const uint32_t w[8]) {
  for (int i = 0; i < 8; ++i) for (int j = 0; j < 4; ++j) b[4 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

// Non-uniform plan exercised on the host: 14 positions of 7 bits + 26 of 6 bits
// (14*7 + 26*6 = 254, the balanced shape of the GPU's plans, incl. take_last).
using PLAN_H = plan<40, 6, 14>;

// Table of plan PL: position bases by repeated doubling, entries by repeated
// addition (independent of comb_entry, which the w = 4 tables still use).
template <class PL>
static void build_table_incremental(const ge& P0, uint32_t* out) {
  ge base = P0;
  for (int pos = 0; pos < PL::P; ++pos) {
    if (pos > 0)
      for (int i = 0; i < PL::width(pos - 1); ++i) ge_dbl(base, base);
    niels n;
    niels_identity(n);
    store_niels(out + (size_t)PL::offset(pos) * 32, n);
    ge acc = base;
    for (uint32_t j = 1; j < PL::entries(pos); ++j) {
      ge_to_niels(n, acc);
      store_niels(out + ((size_t)PL::offset(pos) + j) * 32, n);
      ge t;
      ge_add(t, acc, base);
      acc = t;
    }
  }
}

template <int W>
static void build_table(const ge& P0, uint32_t* out) {
  for (int pos = 0; pos < comb<W>::P; ++pos)
    for (int j = 0; j < (int)comb<W>::E; ++j) {
      niels n;
      comb_entry<comb<W>>(n, P0, pos, j);
      store_niels(out + ((size_t)pos * comb<W>::E + j) * 32, n);
    }
}

static const ds_table g_ds_tab;


// Host emulation of fe_invert_wave (inv25519.h): the same per-lane arithmetic over one 16-lane row, the DPP
// row shifts and readlanes spelled out -- checks the algorithm and its limb bounds off the GPU.
static void fe_invert_wave_emu(fe& out, const fe& z, int* batches = nullptr) {
  uint32_t w[8];
  fe_to_words(w, z);
  int32_t f[16], g[16], D[16], E[16];
  for (int li = 0; li < 16; ++li) {
    g[li] = 0;
    if (li < 9) {
      const int b = 30 * li, wi = b >> 5, sh = b & 31;
      uint64_t x = w[wi] >> sh;
      if (wi + 1 < 8) x |= (uint64_t)w[wi + 1] << (32 - sh);
      g[li] = (int32_t)((uint32_t)x & INV_M30);
    }
    f[li] = li == 0 ? 0x3FFFFFED : li < 8 ? 0x3FFFFFFF : li == 8 ? 0x7FFF : 0;
    D[li] = 0; E[li] = li == 0 ? 1 : 0;
  }
  auto below = [](const int32_t* x, int li) { return li == 0 ? 0 : x[li - 1]; };
  auto above = [](const int32_t* x, int li) { return li == 15 ? 0 : x[li + 1]; };
  int32_t zeta = -1;
  int k = 0;
  for (; k < 20; ++k) {
    bool any = false;
    for (int li = 0; li < 16; ++li) any |= g[li] != 0;
    if (!any) break;
    int32_t t[4];
    zeta = divsteps30_tab(zeta, (uint32_t)f[0], (uint32_t)g[0], t, g_ds_tab.e);
    const int64_t u = t[0], v = t[1], q = t[2], r = t[3];
    int32_t lf[16], lg[16], hf[16], hg[16], nf[16], ng[16], cf[16], cg[16];
    for (int li = 0; li < 16; ++li) {
      const int64_t af = u * f[li] + v * g[li], ag = q * f[li] + r * g[li];
      if (af > ((int64_t)1 << 62) || af < -((int64_t)1 << 62)) throw 1;
      lf[li] = (int32_t)((uint32_t)af & INV_M30); lg[li] = (int32_t)((uint32_t)ag & INV_M30);
      hf[li] = (int32_t)(af >> 30); hg[li] = (int32_t)(ag >> 30);
    }
    for (int li = 0; li < 16; ++li) {
      nf[li] = hf[li] + above(lf, li); ng[li] = hg[li] + above(lg, li);
      const int32_t fc = li < 8 ? -1 : 0;
      cf[li] = (nf[li] >> 30) & fc; cg[li] = (ng[li] >> 30) & fc;
    }
    for (int li = 0; li < 16; ++li) {
      const uint32_t fm = li < 8 ? INV_M30 : 0xFFFFFFFFu;
      f[li] = (int32_t)((uint32_t)nf[li] & fm) + below(cf, li);
      g[li] = (int32_t)((uint32_t)ng[li] & fm) + below(cg, li);
    }
    int64_t ad[16], ae[16], nd[16], ne[16];
    int32_t hd[16], he[16], kd[16], ke[16];
    for (int li = 0; li < 16; ++li) {
      const int dsh = (li & 1) ? 25 : 26;
      ad[li] = u * D[li] + v * E[li]; ae[li] = q * D[li] + r * E[li];
      const int64_t hd64 = ad[li] >> dsh, he64 = ae[li] >> dsh;
      if (hd64 != (int32_t)hd64 || he64 != (int32_t)he64) throw 2;
      hd[li] = (int32_t)hd64; he[li] = (int32_t)he64;
    }
    for (int li = 0; li < 16; ++li) {
      const int dsh = (li & 1) ? 25 : 26;
      const uint32_t dm = (1u << dsh) - 1u;
      const int32_t w19 = li == 0 ? 19 : 0;
      const int64_t sd = (int64_t)((uint32_t)ad[li] & dm) + below(hd, li), se = (int64_t)((uint32_t)ae[li] & dm) + below(he, li);
      if (sd != (int32_t)sd || se != (int32_t)se) throw 3;
      nd[li] = sd + (int64_t)w19 * hd[9]; ne[li] = se + (int64_t)w19 * he[9];
      const int64_t kd64 = nd[li] >> dsh, ke64 = ne[li] >> dsh;
      if (kd64 != (int32_t)kd64 || ke64 != (int32_t)ke64) throw 4;
      kd[li] = (int32_t)kd64; ke[li] = (int32_t)ke64;
    }
    for (int li = 0; li < 16; ++li) {
      const int dsh = (li & 1) ? 25 : 26;
      const uint32_t dm = (1u << dsh) - 1u;
      const int32_t w19 = li == 0 ? 19 : 0, dl = li < 10 ? -1 : 0;
      D[li] = ((int32_t)((uint32_t)nd[li] & dm) + below(kd, li) + w19 * kd[9]) & dl;
      E[li] = ((int32_t)((uint32_t)ne[li] & dm) + below(ke, li) + w19 * ke[9]) & dl;
      if (D[li] > (1 << 26) + (1 << 12) || D[li] < -(1 << 12) || E[li] > (1 << 26) + (1 << 12) || E[li] < -(1 << 12))
        throw 5;
    }
  }
  if (batches) *batches = k;
  const bool neg = ((uint32_t)f[0] & INV_M30) != 1u;
  fe d, c, p2;
  for (int i = 0; i < 10; ++i) {
    d.v[i] = (uint32_t)D[i] + (i == 0 ? 0x7FFFFDAu : (i & 1) ? 0x3FFFFFEu : 0x7FFFFFEu);
    c.v[i] = DS_INV2K[k][i];
  }
  fe_mul(out, d, c);
  if (neg) { fe_neg(p2, out); fe_carry(p2); out = p2; }
}

extern "C" {

// divsteps30_tab against divsteps30 on n pseudo-random (zeta, f odd, g) triples: number of mismatches
int hh_divsteps_tab_check(uint64_t seed, int n) {
  int bad = 0;
  uint64_t x = seed;
  auto next = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
  for (int i = 0; i < n; ++i) {
    const uint64_t a = next(), b = next();
    int32_t zeta = (int32_t)(a % 41) - 20;  // zeta classes well past the clamp on both sides
    if (i % 7 == 0) zeta = (int32_t)(b % 1200) - 600;
    const uint32_t f = (uint32_t)(a >> 32) | 1u, g = (uint32_t)b;
    int32_t t1[4], t2[4];
    const int32_t z1 = divsteps30(zeta, f, g, t1), z2 = divsteps30_tab(zeta, f, g, t2, g_ds_tab.e);
    bad += (z1 != z2 || t1[0] != t2[0] || t1[1] != t2[1] || t1[2] != t2[2] || t1[3] != t2[3]);
  }
  return bad;
}

void hh_fe_op(int op, const uint8_t* a, const uint8_t* b, uint8_t* out) {
  uint32_t wa[8], wb[8], wo[8];
  words_from_bytes(wa, a); words_from_bytes(wb, b);
  fe fa, fb, fo;
  fe_from_words(fa, wa); fe_from_words(fb, wb);
  switch (op) {
    case 0: fe_mul(fo, fa, fb); break;
    case 1: fe_sq(fo, fa); break;
    case 2: fe_invert(fo, fa); break;
    case 3: fe_pow22523(fo, fa); break;
    case 4: { fe t; fe_add(t, fa, fb); fe_mul(fo, t, t); break; }     // (a+b)^2 via mul of unreduced
    case 5: { fe t; fe_sub(t, fa, fb); fe_mul(fo, t, fb); break; }    // (a-b)*b
    case 6: { fe t; fe_add(t, fa, fb); fe_sq(fo, t); break; }         // (a+b)^2 via sq of unreduced
    // latency-oriented (parallel-carry) variants
    case 7: fe_mulT<true>(fo, fa, fb); break;
    case 8: fe_sqT<true>(fo, fa); break;
    case 9: fe_invert<true>(fo, fa); break;
    case 10: fe_pow22523<true>(fo, fa); break;
    case 11: { fe t; fe_add(t, fa, fb); fe_mulT<true>(fo, t, t); break; }
    case 12: { fe t; fe_sub(t, fa, fb); fe_mulT<true>(fo, t, fb); break; }
    case 13: { fe t, u; fe_sqT<true>(t, fa); fe_sub(u, fb, t); fe_mulT<true>(fo, u, t); break; }  // par output as subtrahend
    case 14: fe_invert_gcd(fo, fa); break;                            // safegcd (divsteps) inversion
    case 15: { fe t; fe_add(t, fa, fb); fe_invert_gcd(fo, t); break; } // of an uncarried sum
    case 16: fe_invert_var(fo, fa); break;                            // variable-time divsteps (uniform input)
    case 17: { fe t; fe_add(t, fa, fb); fe_invert_var(fo, t); break; }
    case 18: fe_invert_tab(fo, fa, g_ds_tab.e); break;                // table-driven divsteps (uniform input)
    case 19: { fe t; fe_add(t, fa, fb); fe_invert_tab(fo, t, g_ds_tab.e); break; }
    case 20: try { fe_invert_wave_emu(fo, fa); } catch (int e) { fe_zero(fo); fo.v[0] = 1000u + (uint32_t)e; } break;
    case 21: { fe t; fe_add(t, fa, fb); try { fe_invert_wave_emu(fo, t); } catch (int e) { fe_zero(fo); fo.v[0] = 1000u + (uint32_t)e; } break; }
    default: fo = fa;
  }
  fe_to_words(wo, fo);
  bytes_from_words(out, wo);
}

// fixed_len: use the compile-time-length specialisation (constant padding words, peeled last block) the
// kernels instantiate, for the lengths listed; otherwise the runtime-length form
void hh_sha512_ram(const uint8_t* r, const uint8_t* a, const uint8_t* m, int len, uint8_t* out64, int fixed_len) {
  uint32_t wr[8], wa[8], h[16];
  words_from_bytes(wr, r); words_from_bytes(wa, a);
  switch (fixed_len ? len : -1) {
    case 0: sha512_ram<0>(h, wr, wa, m, len); break;
    case 47: sha512_ram<47>(h, wr, wa, m, len); break;
    case 48: sha512_ram<48>(h, wr, wa, m, len); break;
    case 85: sha512_ram<85>(h, wr, wa, m, len); break;
    case 111: sha512_ram<111>(h, wr, wa, m, len); break;
    case 112: sha512_ram<112>(h, wr, wa, m, len); break;
    case 240: sha512_ram<240>(h, wr, wa, m, len); break;
    default: sha512_ram<-1>(h, wr, wa, m, len);
  }
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 4; ++j) out64[4 * i + j] = (uint8_t)(h[i] >> (8 * j));
}

// the votes form's hash: block-2 schedule of the 85-byte envelope once (sha512_env_sched), then per signature
void hh_sha512_ram_env(const uint8_t* r, const uint8_t* a, const uint8_t* m, uint8_t* out64) {
  uint32_t wr[8], wa[8], h[16];
  uint64_t wk[SHA_ENV_WORDS];
  words_from_bytes(wr, r); words_from_bytes(wa, a);
  sha512_env_sched(wk, m);
  sha512_ram_env(h, wr, wa, m, wk);
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 4; ++j) out64[4 * i + j] = (uint8_t)(h[i] >> (8 * j));
}

// sha512_ram85 without the per-envelope table (the per-lane schedule path)
void hh_sha512_ram85(const uint8_t* r, const uint8_t* a, const uint8_t* m, uint8_t* out64) {
  uint32_t wr[8], wa[8], h[16];
  words_from_bytes(wr, r); words_from_bytes(wa, a);
  sha512_ram85(h, wr, wa, m, nullptr);
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 4; ++j) out64[4 * i + j] = (uint8_t)(h[i] >> (8 * j));
}

void hh_reduce512(const uint8_t* x64, uint8_t* out32) {
  uint32_t x[16], o[8];
  for (int i = 0; i < 16; ++i) x[i] = x64[4 * i] | (x64[4 * i + 1] << 8) | (x64[4 * i + 2] << 16) | ((uint32_t)x64[4 * i + 3] << 24);
  sc_reduce512(o, x);
  bytes_from_words(out32, o);
}

// decompress + small-order (returns 0 bad encoding, 1 ok, 2 small order)
int hh_decompress(const uint8_t* enc, uint8_t* out_compressed) {
  uint32_t w[8];
  words_from_bytes(w, enc);
  ge p, q;
  const bool ok = ge_decompress(p, w);
  if (ok != ge_decompress<true>(q, w)) return -1;  // the latency-oriented form must agree
  if (!ok) return 0;
  uint32_t a[8], b[8];
  for (int c = 0; c < 2; ++c) {
    fe_to_words(a, c ? p.X : p.Y); fe_to_words(b, c ? q.X : q.Y);
    for (int i = 0; i < 8; ++i) if (a[i] != b[i]) return -1;
  }
  fe zi, x, y;
  fe_invert(zi, p.Z); fe_mul(x, p.X, zi); fe_mul(y, p.Y, zi);
  uint32_t xw[8], yw[8];
  fe_to_words(xw, x); fe_to_words(yw, y);
  yw[7] |= (xw[0] & 1u) << 31;
  bytes_from_words(out_compressed, yw);
  return ge_is_small_order(p) ? 2 : 1;
}

static int table_words(int w) {
  switch (w) { case 4: return (int)comb<4>::TABLE_WORDS; case 5: return (int)comb<5>::TABLE_WORDS;
               case 6: return (int)comb<6>::TABLE_WORDS; case 8: return (int)comb<8>::TABLE_WORDS;
               case 67: return (int)PLAN_H::TABLE_WORDS; }
  return -1;
}
int hh_table_words(int w) { return table_words(w); }

// comb table of (negate ? -P : P) for the point encoded by enc; returns 0 on bad encoding
int hh_build_table(int w, const uint8_t* enc, int negate, uint32_t* out) {
  uint32_t e[8];
  words_from_bytes(e, enc);
  ge P;
  if (!ge_decompress(P, e)) return 0;
  if (negate) { ge t; ge_neg(t, P); P = t; }
  switch (w) {
    case 4: build_table<4>(P, out); break;
    case 5: build_table<5>(P, out); break;
    case 6: build_table<6>(P, out); break;
    case 8: build_table<8>(P, out); break;
    case 67: build_table_incremental<PLAN_H>(P, out); break;
    default: return -1;
  }
  return 1;
}

// SoA batch verify on the host with tables from hh_build_table (w = 4 or 8 both sides)
int hh_verify_batch(int w, const uint32_t* tabB, const uint32_t* tabA_all, const uint8_t* keys,
                    const uint8_t* key_ok, uint32_t n_keys, const uint8_t* R, const uint8_t* S,
                    const uint16_t* key_idx, const uint8_t* msg, uint32_t msg_len, uint32_t msg_stride,
                    uint64_t N, uint8_t* accept) {
  const int tw = table_words(w);
  for (uint64_t i = 0; i < N; ++i) {
    uint32_t r[8], s[8], a[8];
    words_from_bytes(r, R + 32 * i); words_from_bytes(s, S + 32 * i);
    uint32_t ki = key_idx[i];
    bool kok = ki < n_keys && key_ok[ki];
    if (ki >= n_keys) ki = 0;
    words_from_bytes(a, keys + 32 * (size_t)ki);
    const uint32_t* tA = tabA_all + (size_t)ki * tw;
    bool ok;
    if (w == 4) ok = verify_lane<comb<4>, comb<4>, -1>(r, s, a, kok, msg + (size_t)msg_stride * i, (int)msg_len, tabB, tA);
    else if (w == 8) ok = verify_lane<comb<8>, comb<8>, -1>(r, s, a, kok, msg + (size_t)msg_stride * i, (int)msg_len, tabB, tA);
    else if (w == 67) ok = verify_lane<PLAN_H, PLAN_H, -1>(r, s, a, kok, msg + (size_t)msg_stride * i, (int)msg_len, tabB, tA);
    else return -1;
    accept[i] = ok;
  }
  return 0;
}

}  // extern "C"

extern "C" int hh_comb2(int w, const uint32_t* tabB, const uint32_t* tabA, const uint8_t* s32, const uint8_t* k32,
                        uint8_t* out_compressed) {
  if (w != 4) return -1;
  uint32_t s[8], k[8];
  words_from_bytes(s, s32); words_from_bytes(k, k32);
  ge P; ge_identity(P);
  digits ds; ds.init(s);
  digits dk; dk.init(k);
  for (int i = 0; i < comb<4>::P; ++i) {
    int d = i + 1 < comb<4>::P ? ds.take<4>() : ds.take_last<4>(); int ad = d < 0 ? -d : d; niels q;
    load_niels(q, tabB + ((size_t)i * comb<4>::E + ad) * 32); ge_madd_signed(P, P, q, d < 0);
    d = i + 1 < comb<4>::P ? dk.take<4>() : dk.take_last<4>(); ad = d < 0 ? -d : d;
    load_niels(q, tabA + ((size_t)i * comb<4>::E + ad) * 32); ge_madd_signed(P, P, q, d < 0);
  }
  fe zi, x, y; fe_invert(zi, P.Z); fe_mul(x, P.X, zi); fe_mul(y, P.Y, zi);
  uint32_t xw[8], yw[8]; fe_to_words(xw, x); fe_to_words(yw, y);
  yw[7] |= (xw[0] & 1u) << 31;
  bytes_from_words(out_compressed, yw);
  return 0;
}

// ---- guard-page check of the comb gathers (VERDICT r01 "What's weak" item 2) ----
// The base-point and key tables are placed so that their last byte is the last
// byte before a PROT_NONE page: any gather past the end of a table faults.
struct guarded {
  void* map = nullptr;
  size_t len = 0;
  uint32_t* p = nullptr;
  explicit guarded(size_t bytes) {
    const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
    const size_t body = (bytes + pg - 1) / pg * pg;
    len = body + pg;
    map = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (map == MAP_FAILED) { map = nullptr; return; }
    mprotect((uint8_t*)map + body, pg, PROT_NONE);
    p = (uint32_t*)((uint8_t*)map + body - bytes);
  }
  ~guarded() { if (map) munmap(map, len); }
};

// verify_lane (the product's per-lane check, plan<40,6,14>) over a batch under
// ONE key, both tables guarded.  unclamped_probe = 1: instead walk the raw
// digits of every s (no s < L clamp, the r01 code path) and touch each table
// entry they select -- the negative control that shows the guard page works.
extern "C" int hh_guard_verify(const uint8_t* key, const uint8_t* R, const uint8_t* S, const uint8_t* msg,
                               uint32_t msg_len, uint32_t msg_stride, uint64_t N, uint8_t* accept,
                               int unclamped_probe) {
  const size_t tb = PLAN_H::TABLE_WORDS * 4;
  guarded gB(tb), gA(tb);
  if (!gB.p || !gA.p) return -2;
  static const uint8_t Benc[32] = {0x58, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                   0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                   0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66};
  uint32_t e[8];
  ge P;
  words_from_bytes(e, Benc);
  if (!ge_decompress(P, e)) return -3;
  build_table_incremental<PLAN_H>(P, gB.p);
  words_from_bytes(e, key);
  const bool kdec = ge_decompress(P, e);
  const bool kok = kdec && !ge_is_small_order(P);
  if (kdec) { ge t; ge_neg(t, P); P = t; } else ge_identity(P);
  build_table_incremental<PLAN_H>(P, gA.p);
  volatile uint32_t sink = 0;  // keeps the probe's loads
  for (uint64_t i = 0; i < N; ++i) {
    uint32_t r[8], s[8];
    words_from_bytes(r, R + 32 * i);
    words_from_bytes(s, S + 32 * i);
    if (unclamped_probe) {
      digits ds;
      ds.init(s);
      static_for<PLAN_H::P>([&](auto ic) {
        constexpr int j = decltype(ic)::value;
        const int d = ds.template take_pos<PLAN_H, j>();
        const int ad = d < 0 ? -d : d;
        niels q;
        load_niels(q, gB.p + ((size_t)PLAN_H::offset(j) + ad) * 32);
        sink ^= q.hpx.v[0];
      });
      accept[i] = 0;
    } else {
      accept[i] = verify_lane<PLAN_H, PLAN_H, -1>(r, s, e, kok, msg + (size_t)msg_stride * i, (int)msg_len, gB.p,
                                                  gA.p);
    }
  }
  (void)sink;
  return 0;
}
