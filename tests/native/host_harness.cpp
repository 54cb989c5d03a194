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

extern "C" {

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
