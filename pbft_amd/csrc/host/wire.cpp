// Wire codec of the PBFT messages feeding the GPU verifier (include/pbft_wire.h):
// UviBytes framing (src/protocol_config.rs:41-129) + serde_json encoding of the
// reference's externally tagged Message enum (src/message.rs:7-31), extended
// with the signed-envelope fields "replica" and "signature".
//
// The decoder mirrors serde_json's acceptance rules for these structs: any
// field order and JSON whitespace, unknown fields skipped, duplicate or missing
// fields rejected, u64 numbers without sign / fraction / exponent / leading
// zeros, strings with the JSON escapes (surrogate pairs combined, lone
// surrogates rejected), input must be valid UTF-8 (String::from_utf8 at
// src/message.rs:17).  The reference panics on any of these errors (.unwrap());
// this codec returns PBFT_EINVAL / a per-frame status instead.
#include "../../../include/pbft_wire.h"

#include <stdio.h>
#include <string.h>
#if defined(__SSE2__)
#include <emmintrin.h>
#endif

#include "../../../include/pbft_replica.h"

namespace {

const char HEX[] = "0123456789abcdef";

// ------------------------------------------------------------------ writer
struct Out {
  char* p;
  size_t cap, n = 0;
  void put(char c) {
    if (n < cap) p[n] = c;
    ++n;
  }
  void puts(const char* s) {
    while (*s) put(*s++);
  }
  void u64(uint64_t v) {
    char b[24];
    int k = 0;
    do { b[k++] = (char)('0' + v % 10); v /= 10; } while (v);
    while (k) put(b[--k]);
  }
  void hex(const uint8_t* b, size_t n_) {
    put('"');
    for (size_t i = 0; i < n_; ++i) { put(HEX[b[i] >> 4]); put(HEX[b[i] & 15]); }
    put('"');
  }
  // serde_json string escaping: " \ and control characters (\b \f \n \r \t, else \u00xx)
  void str(const char* s, size_t len) {
    put('"');
    for (size_t i = 0; i < len; ++i) {
      const unsigned char c = (unsigned char)s[i];
      switch (c) {
        case '"': puts("\\\""); break;
        case '\\': puts("\\\\"); break;
        case '\b': puts("\\b"); break;
        case '\f': puts("\\f"); break;
        case '\n': puts("\\n"); break;
        case '\r': puts("\\r"); break;
        case '\t': puts("\\t"); break;
        default:
          if (c < 0x20) { puts("\\u00"); put(HEX[c >> 4]); put(HEX[c & 15]); }
          else put((char)c);
      }
    }
    put('"');
  }
};

void write_client_request(Out& o, const pbft_wire_msg* m) {
  o.puts("{\"operation\":");
  o.str(m->operation ? m->operation : "", m->operation ? m->operation_len : 0);
  o.puts(",\"timestamp\":");
  o.u64(m->timestamp);
  o.puts(",\"client\":");
  o.str(m->client, strnlen(m->client, sizeof m->client));
  o.put('}');
}

// ------------------------------------------------------------------ parser
// (r06: the frames are ASCII but for an operation's text -- 8 bytes per step while no byte has its top bit set)
static inline uint64_t load8(const void* p) {
  uint64_t w;
  memcpy(&w, p, 8);
  return w;
}
bool utf8_valid(const unsigned char* s, size_t n) {
  size_t i = 0;
  while (i < n) {
    while (n - i >= 8 && !(load8(s + i) & 0x8080808080808080ull)) i += 8;
    if (i >= n) break;
    const unsigned char c = s[i];
    if (c < 0x80) { ++i; continue; }
    int k;
    uint32_t cp;
    if ((c & 0xE0) == 0xC0) { k = 1; cp = c & 0x1F; }
    else if ((c & 0xF0) == 0xE0) { k = 2; cp = c & 0x0F; }
    else if ((c & 0xF8) == 0xF0) { k = 3; cp = c & 0x07; }
    else return false;
    if (i + (size_t)k >= n) return false;
    for (int j = 1; j <= k; ++j) {
      if ((s[i + j] & 0xC0) != 0x80) return false;
      cp = (cp << 6) | (s[i + j] & 0x3F);
    }
    if ((k == 1 && cp < 0x80) || (k == 2 && cp < 0x800) || (k == 3 && cp < 0x10000)) return false;  // overlong
    if (cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return false;
    i += (size_t)k + 1;
  }
  return true;
}

struct Parser {
  Parser(const char* b, const char* e_, char* a, size_t c) : p(b), e(e_), arena(a), cap(c) {}
  const char* p;
  const char* e;
  char* arena;
  size_t cap, used = 0;

  void ws() {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  bool lit(char c) {
    ws();
    if (p < e && *p == c) { ++p; return true; }
    return false;
  }
  bool emit(char c) {
    if (!arena || used >= cap) return false;
    arena[used++] = c;
    return true;
  }
  bool emit_cp(uint32_t cp) {
    if (cp < 0x80) return emit((char)cp);
    if (cp < 0x800) return emit((char)(0xC0 | (cp >> 6))) && emit((char)(0x80 | (cp & 0x3F)));
    if (cp < 0x10000)
      return emit((char)(0xE0 | (cp >> 12))) && emit((char)(0x80 | ((cp >> 6) & 0x3F))) &&
             emit((char)(0x80 | (cp & 0x3F)));
    return emit((char)(0xF0 | (cp >> 18))) && emit((char)(0x80 | ((cp >> 12) & 0x3F))) &&
           emit((char)(0x80 | ((cp >> 6) & 0x3F))) && emit((char)(0x80 | (cp & 0x3F)));
  }
  bool hex4(uint32_t* v) {
    if (e - p < 4) return false;
    uint32_t x = 0;
    for (int i = 0; i < 4; ++i) {
      const char c = p[i];
      x <<= 4;
      if (c >= '0' && c <= '9') x |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') x |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') x |= (uint32_t)(c - 'A' + 10);
      else return false;
    }
    p += 4;
    *v = x;
    return true;
  }
  // The bytes of a string up to its closing quote when it has no escape or control character: 8 per step (SWAR:
  // a byte equal to '"' or '\\', or below 0x20, stops the word loop), then byte by byte; q = where it stopped.
  static inline bool special8(uint64_t w) {
    constexpr uint64_t ones = 0x0101010101010101ull, high = 0x8080808080808080ull;
    const uint64_t quote = w ^ (ones * '"'), bslash = w ^ (ones * '\\');
    return (((quote - ones) & ~quote) | ((bslash - ones) & ~bslash) | ((w - ones * 0x20) & ~w)) & high;
  }
  const char* plain_end(const char* q) const {
    while (e - q >= 8 && !special8(load8(q))) q += 8;
    while (q < e && *q != '"' && *q != '\\' && (unsigned char)*q >= 0x20) ++q;
    return q;
  }
  // A string in place (no copy) when it has no escape -- the keys, the hex digest and signature; else unescaped into
  // the arena (the caller restores `used` after reading it).
  bool view(const char** s, size_t* n) {
    ws();
    if (p >= e || *p != '"') return false;
    const char* q = plain_end(p + 1);
    if (q < e && *q == '"') {
      *s = p + 1;
      *n = (size_t)(q - p - 1);
      p = q + 1;
      return true;
    }
    return str(s, n, true);
  }
  // string -> arena (store=true) or validated and skipped; *s/*n describe the unescaped bytes
  bool str(const char** s, size_t* n, bool store) {
    ws();
    if (p >= e || *p != '"') return false;
    ++p;
    const size_t start = used;
    {  // the common case: no escape -- one copy
      const char* q = plain_end(p);
      if (q < e && *q == '"') {
        const size_t k = (size_t)(q - p);
        if (store) {
          if (!arena || cap - used < k) return false;
          memcpy(arena + used, p, k);
          used += k;
        }
        p = q + 1;
        if (s) *s = store ? arena + start : nullptr;
        if (n) *n = k;
        return true;
      }
    }
    while (true) {
      if (p >= e) return false;
      const unsigned char c = (unsigned char)*p++;
      if (c == '"') break;
      if (c < 0x20) return false;
      if (c != '\\') {
        if (store && !emit((char)c)) return false;
        continue;
      }
      if (p >= e) return false;
      const char x = *p++;
      char o;
      switch (x) {
        case '"': o = '"'; break;
        case '\\': o = '\\'; break;
        case '/': o = '/'; break;
        case 'b': o = '\b'; break;
        case 'f': o = '\f'; break;
        case 'n': o = '\n'; break;
        case 'r': o = '\r'; break;
        case 't': o = '\t'; break;
        case 'u': {
          uint32_t cp;
          if (!hex4(&cp)) return false;
          if (cp >= 0xDC00 && cp <= 0xDFFF) return false;  // lone low surrogate
          if (cp >= 0xD800 && cp <= 0xDBFF) {
            uint32_t lo;
            if (e - p < 6 || p[0] != '\\' || p[1] != 'u') return false;
            p += 2;
            if (!hex4(&lo) || lo < 0xDC00 || lo > 0xDFFF) return false;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          if (store && !emit_cp(cp)) return false;
          continue;
        }
        default: return false;
      }
      if (store && !emit(o)) return false;
    }
    if (s) *s = store ? arena + start : nullptr;
    if (n) *n = used - start;
    return true;
  }
  char kbuf[64];
  bool key(const char** s, size_t* n) {
    // keys are short: in place, or (escaped) unescaped into a private buffer (the caller compares immediately)
    char* a = arena;
    const size_t c = cap, u = used;
    arena = kbuf; cap = sizeof kbuf; used = 0;
    const bool ok = view(s, n);
    arena = a; cap = c; used = u;
    return ok && lit(':');
  }
  bool u64(uint64_t* v) {
    ws();
    if (p >= e || *p < '0' || *p > '9') return false;
    if (*p == '0' && p + 1 < e && p[1] >= '0' && p[1] <= '9') return false;  // leading zero
    uint64_t x = 0;
    while (p < e && *p >= '0' && *p <= '9') {
      const uint64_t d = (uint64_t)(*p - '0');
      if (x > (UINT64_MAX - d) / 10) return false;
      x = x * 10 + d;
      ++p;
    }
    if (p < e && (*p == '.' || *p == 'e' || *p == 'E')) return false;  // a float is not a u64
    *v = x;
    return true;
  }
  bool skip_value(int depth = 0) {
    if (depth > 64) return false;
    ws();
    if (p >= e) return false;
    const char c = *p;
    if (c == '"') return str(nullptr, nullptr, false);
    if (c == '{' || c == '[') {
      const char close = c == '{' ? '}' : ']';
      ++p;
      if (lit(close)) return true;
      while (true) {
        if (c == '{') {
          if (!str(nullptr, nullptr, false) || !lit(':')) return false;
        }
        if (!skip_value(depth + 1)) return false;
        if (lit(',')) continue;
        return lit(close);
      }
    }
    if (c == '-' || (c >= '0' && c <= '9')) {
      ++p;
      while (p < e && ((*p >= '0' && *p <= '9') || *p == '.' || *p == 'e' || *p == 'E' || *p == '+' || *p == '-'))
        ++p;
      return true;
    }
    static const char* const WORDS[3] = {"true", "false", "null"};
    for (const char* w : WORDS) {
      const size_t k = strlen(w);
      if ((size_t)(e - p) >= k && memcmp(p, w, k) == 0) { p += k; return true; }
    }
    return false;
  }
};

bool eq(const char* s, size_t n, const char* lit_) { return strlen(lit_) == n && memcmp(s, lit_, n) == 0; }

// lowercase hex digit values (format!("{:x}") is lowercase), 0xFF for anything else
struct HexTable {
  uint8_t v[256];
  constexpr HexTable() : v() {
    for (int c = 0; c < 256; ++c) v[c] = 0xFF;
    for (int c = '0'; c <= '9'; ++c) v[c] = (uint8_t)(c - '0');
    for (int c = 'a'; c <= 'f'; ++c) v[c] = (uint8_t)(c - 'a' + 10);
  }
};
constexpr HexTable HEX_VAL{};
// 8 lowercase hex characters -> 4 bytes, SWAR; false if any is not one of 0-9a-f.  Per character: value = low
// nibble + 9 if bit 6 is set (letters); valid iff the value is < 16 and maps back to exactly that character.
static inline bool hex8(const char* s, uint32_t* out) {
  constexpr uint64_t ones = 0x0101010101010101ull, high = 0x8080808080808080ull;
  const uint64_t w = load8(s);
  const uint64_t val = (w & (ones * 0x0F)) + ((w >> 6) & ones) * 9;
  const uint64_t gt9 = ((val + ones * 0x76) & high) >> 7;
  const uint64_t recon = val + ones * 0x30 + gt9 * 0x27;
  uint64_t x = ((val & 0x00FF00FF00FF00FFull) << 4) | ((val >> 8) & 0x00FF00FF00FF00FFull);
  x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
  x = (x | (x >> 16)) & 0xFFFFFFFFull;
  *out = (uint32_t)x;
  return recon == w && !((val + ones * 0x70) & high);
}
#if defined(__SSE2__)
// 16 lowercase hex characters -> 8 bytes (one 8-byte store), SSE2 (the x86-64 baseline); the same rule as hex8
static inline bool hex16_sse2(const char* s, uint8_t* out) {
  const __m128i c = _mm_loadu_si128((const __m128i*)s);
  const __m128i letter = _mm_cmpeq_epi8(_mm_and_si128(c, _mm_set1_epi8(0x40)), _mm_set1_epi8(0x40));
  const __m128i val = _mm_add_epi8(_mm_and_si128(c, _mm_set1_epi8(0x0F)), _mm_and_si128(letter, _mm_set1_epi8(9)));
  const __m128i gt9 = _mm_cmpgt_epi8(val, _mm_set1_epi8(9));
  const __m128i recon = _mm_add_epi8(_mm_add_epi8(val, _mm_set1_epi8(0x30)), _mm_and_si128(gt9, _mm_set1_epi8(0x27)));
  const __m128i bad = _mm_or_si128(_mm_xor_si128(_mm_cmpeq_epi8(recon, c), _mm_set1_epi8(-1)),
                                   _mm_cmpgt_epi8(val, _mm_set1_epi8(15)));
  // (byte 2k holds the high nibble of output byte k: 16-bit lanes (lo << 4) | hi, packed to bytes)
  const __m128i pairs = _mm_or_si128(_mm_slli_epi16(_mm_and_si128(val, _mm_set1_epi16(0x00FF)), 4),
                                     _mm_srli_epi16(val, 8));
  _mm_storel_epi64((__m128i*)out, _mm_packus_epi16(pairs, pairs));
  return _mm_movemask_epi8(bad) == 0;
}
#endif
bool parse_hex(const char* s, size_t n, uint8_t* out, size_t nbytes) {
  if (n != 2 * nbytes) return false;
  size_t i = 0;
  bool ok = true;
#if defined(__SSE2__)
  for (; i + 8 <= nbytes; i += 8) ok &= hex16_sse2(s + 2 * i, out + i);
#endif
  // (8 output bytes per store: the digest and signature are read back 8 bytes at a time -- push's compare and row
  // copy -- and 4-byte stores under 8-byte loads would defeat store-to-load forwarding)
  for (; i + 8 <= nbytes; i += 8) {
    uint32_t lo, hi;
    ok &= hex8(s + 2 * i, &lo);
    ok &= hex8(s + 2 * i + 8, &hi);
    const uint64_t v = (uint64_t)lo | (uint64_t)hi << 32;
    memcpy(out + i, &v, 8);
  }
  uint8_t bad = 0;
  for (; i < nbytes; ++i) {
    const uint8_t hi = HEX_VAL.v[(uint8_t)s[2 * i]], lo = HEX_VAL.v[(uint8_t)s[2 * i + 1]];
    bad |= (uint8_t)(hi | lo);
    out[i] = (uint8_t)(hi << 4 | (lo & 15));
  }
  return ok && !(bad & 0x80);  // (every valid digit is < 16: an invalid one sets the top bit)
}

bool parse_client_request(Parser& P, pbft_wire_msg* m) {
  if (!P.lit('{')) return false;
  bool has_op = false, has_ts = false, has_cl = false;
  if (!P.lit('}')) {
    do {
      const char* k;
      size_t kn;
      if (!P.key(&k, &kn)) return false;
      if (eq(k, kn, "operation")) {
        if (has_op) return false;
        const char* s;
        size_t n;
        if (!P.str(&s, &n, true)) return false;
        m->operation = s;
        m->operation_len = (uint32_t)n;
        has_op = true;
      } else if (eq(k, kn, "timestamp")) {
        if (has_ts || !P.u64(&m->timestamp)) return false;
        has_ts = true;
      } else if (eq(k, kn, "client")) {
        if (has_cl) return false;
        const size_t mark = P.used;
        const char* s;
        size_t n;
        if (!P.str(&s, &n, true) || n == 0 || n >= sizeof m->client) return false;
        memcpy(m->client, s, n);
        m->client[n] = 0;
        P.used = mark;
        has_cl = true;
      } else if (!P.skip_value()) {
        return false;
      }
    } while (P.lit(','));
    if (!P.lit('}')) return false;
  }
  return has_op && has_ts && has_cl;
}

bool parse_body(Parser& P, uint32_t kind, pbft_wire_msg* m) {
  if (kind == PBFT_MSG_CLIENT_REQUEST) return parse_client_request(P, m);
  if (!P.lit('{')) return false;
  bool has_v = false, has_n = false, has_d = false, has_m = false, has_r = false, has_s = false;
  if (!P.lit('}')) {
    do {
      const char* k;
      size_t kn;
      if (!P.key(&k, &kn)) return false;
      if (eq(k, kn, "view")) {
        if (has_v || !P.u64(&m->view)) return false;
        has_v = true;
      } else if (eq(k, kn, "sequence_number")) {
        if (has_n || !P.u64(&m->seq)) return false;
        has_n = true;
      } else if (eq(k, kn, "digest")) {
        if (has_d) return false;
        const size_t mark = P.used;
        const char* s;
        size_t n;
        if (!P.view(&s, &n)) return false;
        m->digest_ok = parse_hex(s, n, m->digest, 64) ? 1u : 0u;
        P.used = mark;
        has_d = true;
      } else if (kind == PBFT_MSG_PREPREPARE && eq(k, kn, "message")) {
        if (has_m || !parse_client_request(P, m)) return false;
        has_m = true;
      } else if (eq(k, kn, "replica")) {
        uint64_t r;
        if (has_r || !P.u64(&r) || r > 0xFFFFu) return false;
        m->replica = (uint32_t)r;
        has_r = true;
      } else if (eq(k, kn, "signature")) {
        if (has_s) return false;
        const size_t mark = P.used;
        const char* s;
        size_t n;
        if (!P.view(&s, &n) || !parse_hex(s, n, m->sig, 64)) return false;
        P.used = mark;
        has_s = true;
      } else if (!P.skip_value()) {
        return false;
      }
    } while (P.lit(','));
    if (!P.lit('}')) return false;
  }
  if (has_r != has_s) return false;  // the extension comes as a pair
  m->has_sig = has_s ? 1u : 0u;
  return has_v && has_n && has_d && (kind != PBFT_MSG_PREPREPARE || has_m);
}

// The canonical compact form of a signed vote, exactly as serde_json (and pbft_wire_encode_json) writes it:
//   {"Prepare":{"view":V,"sequence_number":N,"digest":"<128 hex>","replica":R,"signature":"<128 hex>"}}
// (or "Commit") matched byte for byte, numbers and hex decoded in place (r06: the single-message JSON ingress).
// Every byte it accepts is ASCII it checked, so no UTF-8 pass is needed; anything else -- whitespace, another field
// order, an escape, unknown fields, a PrePrepare or an unsigned vote, an invalid number or hex digit -- returns
// false and the general parser decides, with serde's rules, exactly as it did before.
bool fast_vote(const char* s, size_t n, pbft_wire_msg* m) {
  const char* p = s;
  const char* const e = s + n;
  auto lit = [&](const char* L, size_t k) {
    if ((size_t)(e - p) < k || memcmp(p, L, k) != 0) return false;
    p += k;
    return true;
  };
  auto num = [&](uint64_t* v) {  // (the general parser's u64 rules: digits, no leading zero, no overflow)
    if (p >= e || *p < '0' || *p > '9' || (*p == '0' && p + 1 < e && p[1] >= '0' && p[1] <= '9')) return false;
    uint64_t x = 0;
    for (; p < e && *p >= '0' && *p <= '9'; ++p) {
      const uint64_t d = (uint64_t)(*p - '0');
      if (x > (UINT64_MAX - d) / 10) return false;
      x = x * 10 + d;
    }
    *v = x;
    return true;
  };
  auto hex64 = [&](uint8_t* out) {
    if (e - p < 129 || p[128] != '"' || !parse_hex(p, 128, out, 64)) return false;
    p += 129;
    return true;
  };
  uint32_t kind;
  if (lit("{\"Prepare\":{\"view\":", 19)) kind = PBFT_MSG_PREPARE;
  else if (lit("{\"Commit\":{\"view\":", 18)) kind = PBFT_MSG_COMMIT;
  else return false;
  uint64_t view, seq, rep;
  if (!num(&view) || !lit(",\"sequence_number\":", 19) || !num(&seq) || !lit(",\"digest\":\"", 11) ||
      !hex64(m->digest) || !lit(",\"replica\":", 11) || !num(&rep) || rep > 0xFFFFu ||
      !lit(",\"signature\":\"", 14) || !hex64(m->sig) || !lit("}}", 2) || p != e)
    return false;
  m->kind = kind;
  m->view = view;
  m->seq = seq;
  m->digest_ok = 1;
  m->has_sig = 1;
  m->replica = (uint32_t)rep;
  return true;
}

}  // namespace

extern "C" {

size_t pbft_uvi_encode(uint64_t v, uint8_t out[10]) {
  size_t n = 0;
  do {
    uint8_t b = (uint8_t)(v & 0x7F);
    v >>= 7;
    if (v) b |= 0x80;
    out[n++] = b;
  } while (v);
  return n;
}

int pbft_uvi_decode(const uint8_t* buf, size_t len, uint64_t* value, size_t* header_bytes) {
  if (!value || !header_bytes || (!buf && len)) return PBFT_EINVAL;
  uint64_t v = 0;
  for (size_t i = 0; i < 10; ++i) {
    if (i >= len) return 1;  // need more bytes
    const uint8_t b = buf[i];
    if (i == 9 && b > 1) return PBFT_EINVAL;  // > u64
    v |= (uint64_t)(b & 0x7F) << (7 * i);
    if (!(b & 0x80)) {
      if (b == 0 && i > 0) return PBFT_EINVAL;  // non-minimal (unsigned-varint rejects it)
      *value = v;
      *header_bytes = i + 1;
      return 0;
    }
  }
  return PBFT_EINVAL;
}

int pbft_wire_encode_json(const pbft_wire_msg* m, char* out, size_t cap, size_t* len) {
  if (!m || !len || (!out && cap)) return PBFT_EINVAL;
  Out o{out, cap};
  switch (m->kind) {
    case PBFT_MSG_CLIENT_REQUEST:
      o.puts("{\"ClientRequest\":");
      write_client_request(o, m);
      o.put('}');
      break;
    case PBFT_MSG_PREPREPARE:
    case PBFT_MSG_PREPARE:
    case PBFT_MSG_COMMIT:
      o.puts(m->kind == PBFT_MSG_PREPREPARE ? "{\"PrePrepare\":" : m->kind == PBFT_MSG_PREPARE ? "{\"Prepare\":"
                                                                                                : "{\"Commit\":");
      o.puts("{\"view\":");
      o.u64(m->view);
      o.puts(",\"sequence_number\":");
      o.u64(m->seq);
      o.puts(",\"digest\":");
      o.hex(m->digest, 64);
      if (m->kind == PBFT_MSG_PREPREPARE) {
        o.puts(",\"message\":");
        write_client_request(o, m);
      }
      if (m->has_sig) {
        if (m->replica > 0xFFFFu) return PBFT_EINVAL;
        o.puts(",\"replica\":");
        o.u64(m->replica);
        o.puts(",\"signature\":");
        o.hex(m->sig, 64);
      }
      o.puts("}}");
      break;
    default:
      return PBFT_EINVAL;
  }
  *len = o.n;
  return o.n <= cap ? 0 : PBFT_EINVAL;
}

int pbft_wire_encode_frame(const pbft_wire_msg* m, uint8_t* out, size_t cap, size_t* len) {
  if (!len) return PBFT_EINVAL;
  size_t jl = 0;
  const int rc = pbft_wire_encode_json(m, nullptr, 0, &jl);  // length probe
  if (rc && jl == 0) return PBFT_EINVAL;
  if (jl > PBFT_UVI_MAX_FRAME) return PBFT_EINVAL;
  uint8_t hdr[10];
  const size_t hn = pbft_uvi_encode(jl, hdr);
  *len = hn + jl;
  if (!out || cap < hn + jl) return PBFT_EINVAL;
  memcpy(out, hdr, hn);
  return pbft_wire_encode_json(m, (char*)out + hn, jl, &jl);
}

int pbft_wire_decode_json(const char* json, size_t len, pbft_wire_msg* out, char* arena, size_t arena_cap) {
  if (!json || !out) return PBFT_EINVAL;
  memset(out, 0, sizeof *out);
  if (fast_vote(json, len, out)) return 0;
  memset(out, 0, sizeof *out);  // (a partial fast match may have written the digest)
  if (!utf8_valid((const unsigned char*)json, len)) return PBFT_EINVAL;
  Parser P{json, json + len, arena, arena_cap};
  if (!P.lit('{')) return PBFT_EINVAL;
  const char* k;
  size_t kn;
  if (!P.key(&k, &kn)) return PBFT_EINVAL;
  uint32_t kind;
  if (eq(k, kn, "PrePrepare")) kind = PBFT_MSG_PREPREPARE;
  else if (eq(k, kn, "Prepare")) kind = PBFT_MSG_PREPARE;
  else if (eq(k, kn, "Commit")) kind = PBFT_MSG_COMMIT;
  else if (eq(k, kn, "ClientRequest")) kind = PBFT_MSG_CLIENT_REQUEST;
  else return PBFT_EINVAL;
  out->kind = kind;
  if (!parse_body(P, kind, out)) return PBFT_EINVAL;
  if (!P.lit('}')) return PBFT_EINVAL;
  P.ws();
  return P.p == P.e ? 0 : PBFT_EINVAL;  // trailing characters: serde_json errors
}

int pbft_wire_decode_votes(const uint8_t* stream, size_t len, uint32_t n_replicas, uint64_t max_frames,
                           uint64_t max_rows, uint8_t* status, uint8_t* R, uint8_t* S, uint16_t* key_idx,
                           uint8_t* msg, uint8_t* kind, uint64_t* view, uint64_t* seq, uint64_t* n_frames,
                           uint64_t* n_rows, uint64_t* consumed) {
  if (!n_frames || !n_rows || !consumed || (!stream && len)) return PBFT_EINVAL;
  if (max_rows && (!R || !S || !key_idx || !msg)) return PBFT_EINVAL;
  *n_frames = *n_rows = *consumed = 0;
  size_t off = 0;
  // small arena: votes carry no operation; a PrePrepare's operation is parsed
  // (and validated) but only its status is reported here
  static thread_local char arena[1 << 16];
  while (off < len && *n_frames < max_frames && *n_rows < max_rows) {
    uint64_t fl;
    size_t hn;
    const int rc = pbft_uvi_decode(stream + off, len - off, &fl, &hn);
    if (rc == 1) break;
    if (rc != 0 || fl > PBFT_UVI_MAX_FRAME) return PBFT_EINVAL;
    if (len - off - hn < fl) break;  // incomplete frame: keep for the next call
    const char* js = (const char*)stream + off + hn;
    pbft_wire_msg m;
    uint8_t st = PBFT_WIRE_OK;
    if (pbft_wire_decode_json(js, (size_t)fl, &m, arena, sizeof arena) != 0) st = PBFT_WIRE_EJSON;
    else if (m.kind == PBFT_MSG_CLIENT_REQUEST) st = PBFT_WIRE_EKIND;  // signed PrePrepares pass: kind-0 rows
    else if (!m.digest_ok) st = PBFT_WIRE_EDIGEST;
    else if (!m.has_sig) st = PBFT_WIRE_EUNSIGNED;
    else if (m.replica >= n_replicas) st = PBFT_WIRE_ESIGNER;
    if (status) status[*n_frames] = st;
    if (st == PBFT_WIRE_OK) {
      const uint64_t r = (*n_rows)++;
      memcpy(R + 32 * r, m.sig, 32);
      memcpy(S + 32 * r, m.sig + 32, 32);
      key_idx[r] = (uint16_t)m.replica;
      pbft_envelope(msg + PBFT_ENVELOPE_BYTES * r, (uint8_t)m.kind, m.view, m.seq, m.digest);
      if (kind) kind[r] = (uint8_t)m.kind;
      if (view) view[r] = m.view;
      if (seq) seq[r] = m.seq;
    }
    ++*n_frames;
    off += hn + (size_t)fl;
    *consumed = off;
  }
  return 0;
}

int pbft_wire_encode_votes(uint64_t N, const uint8_t* kind, const uint64_t* view, const uint64_t* seq,
                           const uint8_t* digests, const uint32_t* replica, const uint8_t* sigs, uint8_t* out,
                           size_t cap, size_t* len) {
  if (!len || (N && (!kind || !view || !seq || !digests || !replica || !sigs))) return PBFT_EINVAL;
  size_t off = 0;
  int rc = 0;
  for (uint64_t i = 0; i < N; ++i) {
    pbft_wire_msg m;
    memset(&m, 0, sizeof m);
    m.kind = kind[i];
    m.view = view[i];
    m.seq = seq[i];
    memcpy(m.digest, digests + 64 * i, 64);
    m.digest_ok = 1;
    m.has_sig = 1;
    m.replica = replica[i];
    memcpy(m.sig, sigs + 64 * i, 64);
    if (m.kind != PBFT_MSG_PREPARE && m.kind != PBFT_MSG_COMMIT) return PBFT_EINVAL;
    size_t fl = 0;
    const bool room = out && off <= cap;
    const int e = pbft_wire_encode_frame(&m, room ? out + off : nullptr, room ? cap - off : 0, &fl);
    if (fl == 0) return PBFT_EINVAL;
    if (e) rc = PBFT_EINVAL;  // (no room: keep counting the length)
    off += fl;
  }
  *len = off;
  return rc;
}

int pbft_records_pack(const uint8_t* R, const uint8_t* S, const uint16_t* key_idx, const uint8_t* msg,
                      uint32_t msg_stride, uint64_t N, uint8_t* records) {
  if (N && (!R || !S || !key_idx || !msg || !records || msg_stride < PBFT_ENVELOPE_BYTES)) return PBFT_EINVAL;
  for (uint64_t i = 0; i < N; ++i) {
    uint8_t* o = records + PBFT_RECORD_BYTES * i;
    memset(o, 0, PBFT_RECORD_BYTES);
    memcpy(o, R + 32 * i, 32);
    memcpy(o + 32, S + 32 * i, 32);
    memcpy(o + 64, msg + (size_t)msg_stride * i, PBFT_ENVELOPE_BYTES);
    o[150] = (uint8_t)(key_idx[i] & 0xFF);
    o[151] = (uint8_t)(key_idx[i] >> 8);
  }
  return 0;
}

}  // extern "C"
