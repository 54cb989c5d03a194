// Host-side PBFT verification state machine (include/pbft_replica.h): signed
// envelopes, a (view, seq) round batcher that hands ready sub-windows of many
// rounds to the GPU verifier in one batch, the quorum predicates, a
// watermark-bounded log with garbage collection, and the PeerId -> key binding.
//
// Mirrors src/state.rs (State: logs keyed by (view, seq), one vote per peer,
// last write wins :56, :66) and src/behavior.rs (validate_* :126-195, prepared
// :177-182, committed_local :214-223, the caller inject_node_event :304-412)
// with the paper's thresholds (2f, 2f+1), commits keyed by (view, seq) instead of
// view only (src/state.rs:22-23), and the signature checks the reference leaves
// as TODOs (src/behavior.rs:127, :185).
#include <array>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../../include/pbft_replica.h"
#include "../../../include/pbft_wire.h"

namespace {

using Key = std::pair<uint64_t, uint64_t>;  // (view, seq)
using Digest = std::array<uint8_t, 64>;

struct Cand {
  Digest digest;
  uint8_t sig[64];
};

// Votes of one kind in one round window.  Candidates stay pending per signer
// until verified; an accepted vote replaces the signer's previous one
// (HashMap<PeerId, _>::insert in src/state.rs:49-67).
struct Phase {
  std::map<uint32_t, std::vector<Cand>> pending;
  std::map<uint32_t, Digest> accepted;
};

struct Window {
  std::vector<Cand> pp_pending;  // signed PrePrepare candidates (signer = primary of the view)
  bool have_pre_prepare = false;
  Digest digest{};
  Phase ph[2];  // [0] Prepare, [1] Commit
  bool pre_prepared_reported = false, prepared_reported = false, committed_reported = false;
};

}  // namespace

struct pbft_replica {
  pbft_ctx* ctx = nullptr;
  uint32_t n = 0, f = 0, self = 0;
  uint64_t current_view = 1;  // src/view.rs:5-8: the view starts at 1 (no view change)
  uint64_t h = 0;             // low watermark: every seq <= h is done (committed prefix or checkpoint)
  uint64_t h_commit = 0;      // highest seq of the committed prefix
  uint64_t log_window = PBFT_DEFAULT_LOG_WINDOW;
  std::vector<uint8_t> keys;
  std::unordered_map<std::string, uint32_t> key_index;
  std::map<Key, Window> windows;
  std::set<Key> dirty;  // windows whose events must be (re-)evaluated
  pbft_batch_verify_fn verify_fn = nullptr;
  void* verify_user = nullptr;
  pbft_digest_fn digest_fn = nullptr;
  void* digest_user = nullptr;
  pbft_replica_stats stats{};
};

static uint32_t primary_of(const pbft_replica* r, uint64_t view) { return (uint32_t)(view % r->n); }

static bool in_log(const pbft_replica* r, uint64_t seq) { return seq > r->h && seq - r->h <= r->log_window; }

static uint32_t matching(const Window& w, const std::map<uint32_t, Digest>& votes, int64_t exclude = -1) {
  if (!w.have_pre_prepare) return 0;
  uint32_t c = 0;
  for (const auto& kv : votes)
    if ((int64_t)kv.first != exclude && kv.second == w.digest) ++c;
  return c;
}

// prepared(m, v, n, i): pre-prepare + 2f matching prepares from distinct backups
static bool is_prepared(const pbft_replica* r, uint64_t view, const Window& w) {
  return w.have_pre_prepare && matching(w, w.ph[0].accepted, primary_of(r, view)) >= 2 * r->f;
}

// committed-local(m, v, n, i): prepared + 2f+1 matching commits (possibly own)
static bool is_committed_local(const pbft_replica* r, uint64_t view, const Window& w) {
  return is_prepared(r, view, w) && matching(w, w.ph[1].accepted) >= 2 * r->f + 1;
}

// Distinct signers with an accepted or pending vote of this phase (optionally
// excluding one signer, the primary for Prepares).
static uint32_t distinct_signers(const Phase& p, int64_t exclude) {
  uint32_t c = 0;
  for (const auto& kv : p.accepted)
    if ((int64_t)kv.first != exclude) ++c;
  for (const auto& kv : p.pending)
    if ((int64_t)kv.first != exclude && !kv.second.empty() && !p.accepted.count(kv.first)) ++c;
  return c;
}

// A sub-window closes on its own count: enough distinct signers for the quorum
// (2f backups' Prepares / 2f+1 Commits) or every possible signer.
static bool prepare_ready(const pbft_replica* r, uint64_t view, const Window& w) {
  if (w.ph[0].pending.empty() || w.prepared_reported) return false;
  const uint32_t c = distinct_signers(w.ph[0], primary_of(r, view));
  return c >= 2 * r->f || c + 1 >= r->n;
}
static bool commit_ready(const pbft_replica* r, const Window& w) {
  if (w.ph[1].pending.empty() || w.committed_reported) return false;
  const uint32_t c = distinct_signers(w.ph[1], -1);
  return c >= 2 * r->f + 1 || c >= r->n;
}

static std::string key_str(const uint8_t* A) { return std::string((const char*)A, 32); }

static void gc(pbft_replica* r) {
  // committed prefix: h advances over consecutive committed windows of the current view
  for (;;) {
    auto it = r->windows.find({r->current_view, r->h + 1});
    if (it == r->windows.end() || !it->second.committed_reported) break;
    r->dirty.erase(it->first);
    r->windows.erase(it);
    ++r->h;
    r->h_commit = r->h;
    ++r->stats.windows_gc;
  }
  // anything at or below h (stable checkpoint, or stale views)
  for (auto it = r->windows.begin(); it != r->windows.end();) {
    if (it->first.second <= r->h) {
      r->dirty.erase(it->first);
      it = r->windows.erase(it);
      ++r->stats.windows_gc;
    } else {
      ++it;
    }
  }
}

extern "C" {

void pbft_envelope(uint8_t out[PBFT_ENVELOPE_BYTES], uint8_t kind, uint64_t view, uint64_t seq,
                   const uint8_t digest[64]) {
  memcpy(out, "PBFT", 4);
  out[4] = kind;
  for (int i = 0; i < 8; ++i) out[5 + i] = (uint8_t)(view >> (8 * i));
  for (int i = 0; i < 8; ++i) out[13 + i] = (uint8_t)(seq >> (8 * i));
  memcpy(out + 21, digest, 64);
}

int pbft_replica_create(pbft_ctx* ctx, uint32_t n, uint32_t self_id, const uint8_t* keys, pbft_replica** out) {
  if (!out || !keys || n < 1 || n > 65535 || self_id >= n) return PBFT_EINVAL;
  pbft_replica* r = new pbft_replica();
  r->ctx = ctx;
  r->n = n;
  r->f = (n - 1) / 3;
  r->self = self_id;
  r->keys.assign(keys, keys + 32 * (size_t)n);
  for (uint32_t i = 0; i < n; ++i) r->key_index.emplace(key_str(keys + 32 * (size_t)i), i);  // first index wins
  *out = r;
  return PBFT_OK;
}

int pbft_replica_destroy(pbft_replica* r) {
  delete r;
  return PBFT_OK;
}

int pbft_replica_set_verifier(pbft_replica* r, pbft_batch_verify_fn fn, void* user) {
  if (!r) return PBFT_EINVAL;
  r->verify_fn = fn;
  r->verify_user = user;
  return PBFT_OK;
}

int pbft_replica_set_digest_fn(pbft_replica* r, pbft_digest_fn fn, void* user) {
  if (!r) return PBFT_EINVAL;
  r->digest_fn = fn;
  r->digest_user = user;
  return PBFT_OK;
}

int pbft_replica_set_log_window(pbft_replica* r, uint64_t log_window) {
  if (!r || log_window == 0) return PBFT_EINVAL;
  r->log_window = log_window;
  return PBFT_OK;
}

// validate_pre_prepare (src/behavior.rs:126-157) + State::insert_pre_prepare (src/state.rs:40-47);
// the signature (TODO :127) is checked by the next flush, batched with the votes.
int pbft_replica_on_pre_prepare(pbft_replica* r, uint64_t view, uint64_t seq, const uint8_t* op, uint32_t op_len,
                                const uint8_t claimed_digest[64], const uint8_t primary_sig[64],
                                uint8_t digest_out[64]) {
  if (!r || (!op && op_len) || !claimed_digest || !primary_sig) return PBFT_EINVAL;
  uint8_t d[64];
  int rc;
  if (r->digest_fn) {
    rc = r->digest_fn(r->digest_user, op, op_len, d);
  } else {
    if (!r->ctx) return PBFT_ENODEV;
    const uint64_t off = 0;
    const uint8_t empty = 0;
    rc = pbft_digest_blake2b512(r->ctx, op_len ? op : &empty, &off, &op_len, 1, d);
  }
  if (rc) return rc;
  if (digest_out) memcpy(digest_out, d, 64);
  ++r->stats.pushed;
  if (memcmp(d, claimed_digest, 64) != 0) { ++r->stats.rejected_digest; return 0; }  // validate_digest :139-145
  if (view != r->current_view) { ++r->stats.rejected_view; return 0; }                // :134-141
  if (!in_log(r, seq)) { ++r->stats.rejected_watermark; return 0; }                   // h/H TODO :154
  Window& w = r->windows[{view, seq}];
  Cand c;
  memcpy(c.digest.data(), d, 64);
  memcpy(c.sig, primary_sig, 64);
  if (w.have_pre_prepare) {                                                          // :144-151
    if (w.digest != c.digest) ++r->stats.rejected_digest; else ++r->stats.duplicates;
    return 0;
  }
  for (const Cand& o : w.pp_pending)
    if (o.digest == c.digest && memcmp(o.sig, c.sig, 64) == 0) { ++r->stats.duplicates; return 0; }
  if (w.pp_pending.size() >= PBFT_MAX_CANDIDATES) { ++r->stats.dropped_flood; return 0; }
  w.pp_pending.push_back(c);
  return 1;
}

// inject_node_event Prepare / Commit arms (src/behavior.rs:340-412): enqueue into the round window
int pbft_replica_push(pbft_replica* r, uint8_t kind, uint64_t view, uint64_t seq, const uint8_t digest[64],
                      uint32_t signer, const uint8_t sig[64]) {
  if (!r || !digest || !sig || (kind != PBFT_KIND_PREPARE && kind != PBFT_KIND_COMMIT)) return PBFT_EINVAL;
  ++r->stats.pushed;
  if (signer >= r->n || view != r->current_view) { ++r->stats.rejected_view; return 0; }  // validate_commit :187-190
  if (!in_log(r, seq)) { ++r->stats.rejected_watermark; return 0; }
  Window& w = r->windows[{view, seq}];
  if (w.committed_reported) { ++r->stats.duplicates; return 0; }  // late vote for a decided round
  Phase& p = w.ph[kind - 1];
  Cand c;
  memcpy(c.digest.data(), digest, 64);
  memcpy(c.sig, sig, 64);
  auto acc = p.accepted.find(signer);
  if (acc != p.accepted.end() && acc->second == c.digest) { ++r->stats.duplicates; return 0; }
  std::vector<Cand>& cands = p.pending[signer];
  for (const Cand& o : cands)
    if (o.digest == c.digest && memcmp(o.sig, c.sig, 64) == 0) { ++r->stats.duplicates; return 0; }
  if (cands.size() >= PBFT_MAX_CANDIDATES) { ++r->stats.dropped_flood; return 0; }
  cands.push_back(c);
  return 1;
}

int pbft_replica_flush(pbft_replica* r, int force, pbft_round_event* events, uint32_t max_events,
                       uint32_t* n_events) {
  if (!r) return PBFT_EINVAL;
  if (n_events) *n_events = 0;
  // 1. every ready sub-window of every round window -> one SoA batch.  A signer's
  //    candidates travel together, so after the batch none of them is pending.
  struct Row {
    Window* w;
    Key key;
    int kind;  // 0 PrePrepare, 1 Prepare, 2 Commit
    uint32_t signer;
    const Cand* c;
  };
  std::vector<Row> rows;
  for (auto& kv : r->windows) {
    Window& w = kv.second;
    const uint64_t view = kv.first.first;
    for (const Cand& c : w.pp_pending) rows.push_back({&w, kv.first, 0, primary_of(r, view), &c});
    const bool rd[2] = {force || prepare_ready(r, view, w), force || commit_ready(r, w)};
    for (int k = 0; k < 2; ++k) {
      if (!rd[k]) continue;
      for (auto& sc : w.ph[k].pending)
        for (const Cand& c : sc.second) rows.push_back({&w, kv.first, k + 1, sc.first, &c});
    }
  }
  const uint64_t N = rows.size();
  if (N) {
    std::vector<uint8_t> R(32 * N), S(32 * N), M(PBFT_ENVELOPE_BYTES * N + 16, 0);  // + read slack
    std::vector<uint16_t> K(N);
    for (uint64_t i = 0; i < N; ++i) {
      const Row& x = rows[i];
      memcpy(&R[32 * i], x.c->sig, 32);
      memcpy(&S[32 * i], x.c->sig + 32, 32);
      K[i] = (uint16_t)x.signer;
      pbft_envelope(&M[PBFT_ENVELOPE_BYTES * i], (uint8_t)x.kind, x.key.first, x.key.second, x.c->digest.data());
    }
    std::vector<uint64_t> bitmap((N + 63) / 64, 0);
    int rc;
    if (r->verify_fn) {
      rc = r->verify_fn(r->verify_user, R.data(), S.data(), K.data(), M.data(), PBFT_ENVELOPE_BYTES,
                        PBFT_ENVELOPE_BYTES, N, bitmap.data());
    } else {
      if (!r->ctx) return PBFT_ENODEV;
      rc = pbft_verify_batch(r->ctx, R.data(), S.data(), K.data(), M.data(), PBFT_ENVELOPE_BYTES,
                             PBFT_ENVELOPE_BYTES, N, bitmap.data());
    }
    if (rc) return rc;  // nothing applied: the candidates stay pending
    ++r->stats.batches;
    r->stats.verified += N;
    // 2. apply in push order: State::insert_* for accepted votes only (last accepted wins per signer);
    //    the first accepted PrePrepare fixes the window's digest (conflicting ones rejected, :144-151)
    for (uint64_t i = 0; i < N; ++i) {
      const Row& x = rows[i];
      const bool ok = (bitmap[i >> 6] >> (i & 63)) & 1;
      if (!ok) { ++r->stats.rejected_sig; continue; }
      ++r->stats.accepted;
      r->dirty.insert(x.key);
      if (x.kind == 0) {
        if (!x.w->have_pre_prepare) {
          x.w->have_pre_prepare = true;
          x.w->digest = x.c->digest;
        } else if (x.w->digest != x.c->digest) {
          ++r->stats.rejected_digest;
        }
        continue;
      }
      x.w->ph[x.kind - 1].accepted[x.signer] = x.c->digest;
      if (x.w->have_pre_prepare && x.c->digest != x.w->digest) ++r->stats.rejected_digest;
    }
    // 3. drop the verified candidates (the rows point into these vectors: cleared only now)
    for (const Row& x : rows) {
      if (x.kind == 0) x.w->pp_pending.clear();
      else x.w->ph[x.kind - 1].pending.erase(x.signer);
    }
  }
  // 4. events (pre-prepared, prepared :177-182, committed_local :214-223) for every dirty window,
  //    in (view, seq) order; a window stays dirty while an event did not fit into `events`
  uint32_t ne = 0;
  for (auto it = r->dirty.begin(); it != r->dirty.end();) {
    auto wi = r->windows.find(*it);
    if (wi == r->windows.end()) { it = r->dirty.erase(it); continue; }
    Window& w = wi->second;
    const uint64_t view = it->first, seq = it->second;
    bool full = false;
    auto emit = [&](uint32_t kind, bool& reported) {
      if (full) return;
      if (ne >= max_events || !events) { full = true; return; }
      events[ne++] = {view, seq, kind};
      reported = true;
    };
    if (!w.pre_prepared_reported && w.have_pre_prepare) emit(PBFT_EVENT_PRE_PREPARED, w.pre_prepared_reported);
    if (!w.prepared_reported && is_prepared(r, view, w)) emit(PBFT_EVENT_PREPARED, w.prepared_reported);
    if (!w.committed_reported && is_committed_local(r, view, w)) {
      emit(PBFT_EVENT_COMMITTED_LOCAL, w.committed_reported);
      if (w.committed_reported) {  // decided: stragglers are never needed
        w.pp_pending.clear();
        w.ph[0].pending.clear();
        w.ph[1].pending.clear();
      }
    }
    if (full) ++it; else it = r->dirty.erase(it);
  }
  if (n_events) *n_events = ne;
  gc(r);
  return PBFT_OK;
}

// One connection's byte stream of UviBytes/JSON frames (src/protocol_config.rs:50-76 ->
// src/handler.rs:533-548 -> inject_node_event).  peer_idx = the authenticated peer.
int pbft_replica_push_frames(pbft_replica* r, uint32_t peer_idx, const uint8_t* stream, size_t len,
                             uint64_t* consumed, uint64_t* pushed, uint64_t* dropped) {
  if (!r || !consumed || (!stream && len)) return PBFT_EINVAL;
  static thread_local char arena[1 << 16];  // unescaped strings (the PrePrepare's operation)
  uint64_t np = 0, nd = 0;
  size_t off = 0;
  int rc = 0;
  while (off < len) {
    uint64_t fl;
    size_t hn;
    const int u = pbft_uvi_decode(stream + off, len - off, &fl, &hn);
    if (u == 1) break;  // varint incomplete
    if (u != 0 || fl > PBFT_UVI_MAX_FRAME) { rc = PBFT_EINVAL; break; }
    if (len - off - hn < fl) break;  // incomplete frame: keep for the next read
    const char* js = (const char*)stream + off + hn;
    pbft_wire_msg m;
    const bool parsed = pbft_wire_decode_json(js, (size_t)fl, &m, arena, sizeof arena) == 0;
    off += hn + (size_t)fl;
    int got = 0;
    if (!parsed || !m.digest_ok || !m.has_sig) {
      got = 0;  // not a signed PBFT message (the reference would panic in serde_json .unwrap(), src/message.rs:17-18)
    } else if (m.kind == PBFT_MSG_PREPARE || m.kind == PBFT_MSG_COMMIT) {
      // the signer is the authenticated connection (src/behavior.rs:346, :380), never the frame's field
      if (m.replica != peer_idx) ++r->stats.rejected_signer;
      else got = pbft_replica_push(r, (uint8_t)m.kind, m.view, m.seq, m.digest, peer_idx, m.sig);
    } else if (m.kind == PBFT_MSG_PREPREPARE) {
      // signed by the view's primary (the signature proves it; any peer may relay)
      if (r->n == 0 || m.replica != primary_of(r, m.view)) ++r->stats.rejected_signer;
      else
        got = pbft_replica_on_pre_prepare(r, m.view, m.seq, (const uint8_t*)m.operation, m.operation_len, m.digest,
                                          m.sig, nullptr);
    }
    if (got < 0) { rc = got; break; }
    if (got == 1) ++np; else ++nd;
  }
  *consumed = off;
  if (pushed) *pushed = np;
  if (dropped) *dropped = nd;
  return rc;
}

int pbft_replica_stable_checkpoint(pbft_replica* r, uint64_t seq) {
  if (!r) return PBFT_EINVAL;
  if (seq > r->h) r->h = seq;
  gc(r);
  return PBFT_OK;
}

int pbft_replica_prepared(pbft_replica* r, uint64_t view, uint64_t seq) {
  if (!r) return PBFT_EINVAL;
  if (view == r->current_view && seq <= r->h_commit && seq > 0) return 1;  // GC'd committed prefix
  auto it = r->windows.find({view, seq});
  return it != r->windows.end() && is_prepared(r, view, it->second) ? 1 : 0;
}

int pbft_replica_committed_local(pbft_replica* r, uint64_t view, uint64_t seq) {
  if (!r) return PBFT_EINVAL;
  if (view == r->current_view && seq <= r->h_commit && seq > 0) return 1;
  auto it = r->windows.find({view, seq});
  return it != r->windows.end() && is_committed_local(r, view, it->second) ? 1 : 0;
}

int pbft_replica_get_stats(pbft_replica* r, pbft_replica_stats* out) {
  if (!r || !out) return PBFT_EINVAL;
  r->stats.low_watermark = r->h;
  r->stats.live_windows = r->windows.size();
  *out = r->stats;
  return PBFT_OK;
}

// ---- libp2p PeerId <-> Ed25519 key (src/main.rs:39-40; libp2p-core 0.31 identity) ----
static const uint8_t PEER_PREFIX[6] = {0x00, 0x24, 0x08, 0x01, 0x12, 0x20};

int pbft_key_from_peer_id(const uint8_t* peer_id, size_t len, uint8_t A[32]) {
  if (!peer_id || !A || len != PBFT_PEER_ID_BYTES || memcmp(peer_id, PEER_PREFIX, 6) != 0) return PBFT_EINVAL;
  memcpy(A, peer_id + 6, 32);
  return PBFT_OK;
}

void pbft_peer_id_from_key(const uint8_t A[32], uint8_t peer_id[PBFT_PEER_ID_BYTES]) {
  memcpy(peer_id, PEER_PREFIX, 6);
  memcpy(peer_id + 6, A, 32);
}

int pbft_key_from_peer_id_b58(const char* text, size_t len, uint8_t A[32]) {
  static const char ALPHA[] = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";
  if (!text || !A || len == 0 || len > 64) return PBFT_EINVAL;
  uint8_t num[64] = {0};  // big-endian accumulator
  size_t zeros = 0;
  while (zeros < len && text[zeros] == '1') ++zeros;
  for (size_t i = 0; i < len; ++i) {
    const char* p = (const char*)memchr(ALPHA, text[i], 58);
    if (!p || text[i] == '\0') return PBFT_EINVAL;
    uint32_t carry = (uint32_t)(p - ALPHA);
    for (int j = 63; j >= 0; --j) {
      carry += 58u * num[j];
      num[j] = (uint8_t)carry;
      carry >>= 8;
    }
    if (carry) return PBFT_EINVAL;  // longer than 64 bytes
  }
  size_t lead = 0;
  while (lead < 64 && num[lead] == 0) ++lead;
  const size_t body = 64 - lead, total = zeros + body;
  if (total != PBFT_PEER_ID_BYTES) return PBFT_EINVAL;
  uint8_t raw[PBFT_PEER_ID_BYTES] = {0};
  memcpy(raw + zeros, num + lead, body);
  return pbft_key_from_peer_id(raw, PBFT_PEER_ID_BYTES, A);
}

int pbft_replica_peer_index(pbft_replica* r, const uint8_t* peer_id, size_t len) {
  if (!r) return PBFT_EINVAL;
  uint8_t A[32];
  if (pbft_key_from_peer_id(peer_id, len, A) != PBFT_OK) return PBFT_EINVAL;
  auto it = r->key_index.find(key_str(A));
  return it == r->key_index.end() ? PBFT_EINVAL : (int)it->second;
}

}  // extern "C"
