// Host-side PBFT verification state machine (include/pbft_replica.h): signed
// envelopes, a (view, seq) round batcher that hands whole windows to the GPU
// verifier, and the quorum predicates.  Mirrors src/state.rs (State: logs keyed
// by (view, seq), one vote per replica) and src/behavior.rs (validate_* +
// prepared / committed_local), with the paper's thresholds (2f, 2f+1) and
// commits keyed by (view, seq) instead of view only (src/state.rs:22-23).
#include <cstring>
#include <map>
#include <set>
#include <utility>
#include <vector>

#include "../../../include/pbft_replica.h"

namespace {

struct Vote {
  uint8_t kind;
  uint32_t signer;
  uint8_t digest[64];
  uint8_t sig[64];
};

// One (view, seq) round: src/state.rs PrePrepareKey/PrepareKey, plus the batcher.
struct Window {
  bool have_pre_prepare = false;
  uint8_t digest[64] = {0};
  std::vector<Vote> pending;                        // awaiting batch verification
  std::set<std::pair<uint8_t, uint32_t>> pushed;    // (kind, signer) dedup
  uint32_t pushed_prepares = 0, pushed_commits = 0;
  // verified votes by signer -> digest (only digest-matching ones count)
  std::map<uint32_t, std::vector<uint8_t>> prepares, commits;
  bool prepared_reported = false, committed_reported = false;
};

}  // namespace

struct pbft_replica {
  pbft_ctx* ctx = nullptr;
  uint32_t n = 0, f = 0, self = 0;
  uint64_t current_view = 1;  // src/view.rs:5-8: the view starts at 1 (no view change)
  std::vector<uint8_t> keys;
  std::map<std::pair<uint64_t, uint64_t>, Window> windows;
  pbft_batch_verify_fn verify_fn = nullptr;
  void* verify_user = nullptr;
  pbft_digest_fn digest_fn = nullptr;
  void* digest_user = nullptr;
  pbft_replica_stats stats{};
};

static uint32_t primary_of(const pbft_replica* r, uint64_t view) { return (uint32_t)(view % r->n); }

static uint32_t matching(const Window& w, const std::map<uint32_t, std::vector<uint8_t>>& votes,
                         int64_t exclude = -1) {
  if (!w.have_pre_prepare) return 0;
  uint32_t c = 0;
  for (const auto& kv : votes)
    if ((int64_t)kv.first != exclude && memcmp(kv.second.data(), w.digest, 64) == 0) ++c;
  return c;
}

// prepared(m, v, n, i): pre-prepare + 2f matching prepares from distinct backups
static bool is_prepared(const pbft_replica* r, uint64_t view, const Window& w) {
  return w.have_pre_prepare && matching(w, w.prepares, primary_of(r, view)) >= 2 * r->f;
}

// committed-local(m, v, n, i): prepared + 2f+1 matching commits (possibly own)
static bool is_committed_local(const pbft_replica* r, uint64_t view, const Window& w) {
  return is_prepared(r, view, w) && matching(w, w.commits) >= 2 * r->f + 1;
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

// validate_pre_prepare (src/behavior.rs:126-157) + State::insert_pre_prepare (src/state.rs:40-47)
int pbft_replica_on_pre_prepare(pbft_replica* r, uint64_t view, uint64_t seq, const uint8_t* op, uint32_t op_len,
                                const uint8_t claimed_digest[64], uint8_t digest_out[64]) {
  if (!r || (!op && op_len) || !claimed_digest) return PBFT_EINVAL;
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
  if (memcmp(d, claimed_digest, 64) != 0) { ++r->stats.rejected_digest; return 0; }  // validate_digest :139-145
  if (view != r->current_view) { ++r->stats.rejected_view; return 0; }                // :134-141
  Window& w = r->windows[{view, seq}];
  if (w.have_pre_prepare) {                                                          // :144-151
    if (memcmp(w.digest, d, 64) != 0) { ++r->stats.rejected_digest; return 0; }
    return 1;
  }
  w.have_pre_prepare = true;
  memcpy(w.digest, d, 64);
  return 1;
}

// message_to_handler_event (src/handler.rs:533-548) -> the round window
int pbft_replica_push(pbft_replica* r, uint8_t kind, uint64_t view, uint64_t seq, const uint8_t digest[64],
                      uint32_t signer, const uint8_t sig[64]) {
  if (!r || !digest || !sig || (kind != PBFT_KIND_PREPARE && kind != PBFT_KIND_COMMIT)) return PBFT_EINVAL;
  ++r->stats.pushed;
  if (signer >= r->n || view != r->current_view) { ++r->stats.rejected_view; return 0; }  // validate_commit :187-190
  Window& w = r->windows[{view, seq}];
  if (!w.pushed.insert({kind, signer}).second) { ++r->stats.duplicates; return 0; }
  Vote v;
  v.kind = kind;
  v.signer = signer;
  memcpy(v.digest, digest, 64);
  memcpy(v.sig, sig, 64);
  w.pending.push_back(v);
  if (kind == PBFT_KIND_PREPARE) ++w.pushed_prepares; else ++w.pushed_commits;
  return 1;
}

int pbft_replica_flush(pbft_replica* r, int force, pbft_round_event* events, uint32_t max_events,
                       uint32_t* n_events) {
  if (!r) return PBFT_EINVAL;
  if (n_events) *n_events = 0;
  // 1. gather the pending votes of every closed window (all n-1 peers' Prepare and
  //    Commit seen) -- or of every window when forced (deadline) -- into one SoA batch
  std::vector<std::pair<Window*, size_t>> owner;
  std::vector<uint8_t> R, S, M;
  std::vector<uint16_t> K;
  std::vector<std::pair<uint64_t, uint64_t>> keys_of;
  for (auto& kv : r->windows) {
    Window& w = kv.second;
    if (w.pending.empty()) continue;
    const bool closed = w.pushed_prepares + 1 >= r->n && w.pushed_commits + 1 >= r->n;
    if (!closed && !force) continue;
    for (size_t i = 0; i < w.pending.size(); ++i) {
      const Vote& v = w.pending[i];
      R.insert(R.end(), v.sig, v.sig + 32);
      S.insert(S.end(), v.sig + 32, v.sig + 64);
      K.push_back((uint16_t)v.signer);
      uint8_t env[PBFT_ENVELOPE_BYTES];
      pbft_envelope(env, v.kind, kv.first.first, kv.first.second, v.digest);
      M.insert(M.end(), env, env + PBFT_ENVELOPE_BYTES);
      owner.push_back({&w, i});
      keys_of.push_back(kv.first);
    }
  }
  const uint64_t N = K.size();
  if (N == 0) return PBFT_OK;
  M.resize(M.size() + 16, 0);  // read slack for unaligned message loads
  std::vector<uint64_t> bitmap((N + 63) / 64, 0);
  int rc;
  if (r->verify_fn) {
    rc = r->verify_fn(r->verify_user, R.data(), S.data(), K.data(), M.data(), PBFT_ENVELOPE_BYTES,
                      PBFT_ENVELOPE_BYTES, N, bitmap.data());
  } else {
    if (!r->ctx) return PBFT_ENODEV;
    rc = pbft_verify_batch(r->ctx, R.data(), S.data(), K.data(), M.data(), PBFT_ENVELOPE_BYTES, PBFT_ENVELOPE_BYTES,
                           N, bitmap.data());
  }
  if (rc) return rc;
  ++r->stats.batches;
  r->stats.verified += N;
  // 2. State::insert_prepare / insert_commit for accepted votes only
  for (uint64_t i = 0; i < N; ++i) {
    Window* w = owner[i].first;
    const Vote& v = w->pending[owner[i].second];
    if (!((bitmap[i >> 6] >> (i & 63)) & 1)) { ++r->stats.rejected_sig; continue; }
    ++r->stats.accepted;
    auto& log = v.kind == PBFT_KIND_PREPARE ? w->prepares : w->commits;
    log[v.signer] = std::vector<uint8_t>(v.digest, v.digest + 64);
    if (w->have_pre_prepare && memcmp(v.digest, w->digest, 64) != 0) ++r->stats.rejected_digest;
  }
  // 3. quorum predicates (prepared :177-182, committed_local :214-223)
  uint32_t ne = 0;
  std::set<Window*> done;
  for (uint64_t i = 0; i < N; ++i) {
    Window* w = owner[i].first;
    if (!done.insert(w).second) continue;
    w->pending.clear();
    const uint64_t view = keys_of[i].first, seq = keys_of[i].second;
    if (!w->prepared_reported && is_prepared(r, view, *w)) {
      w->prepared_reported = true;
      if (events && ne < max_events) events[ne] = {view, seq, PBFT_EVENT_PREPARED};
      ++ne;
    }
    if (!w->committed_reported && is_committed_local(r, view, *w)) {
      w->committed_reported = true;
      if (events && ne < max_events) events[ne] = {view, seq, PBFT_EVENT_COMMITTED_LOCAL};
      ++ne;
    }
  }
  if (n_events) *n_events = ne < max_events ? ne : max_events;
  return PBFT_OK;
}

int pbft_replica_prepared(pbft_replica* r, uint64_t view, uint64_t seq) {
  if (!r) return PBFT_EINVAL;
  auto it = r->windows.find({view, seq});
  return it != r->windows.end() && is_prepared(r, view, it->second) ? 1 : 0;
}

int pbft_replica_committed_local(pbft_replica* r, uint64_t view, uint64_t seq) {
  if (!r) return PBFT_EINVAL;
  auto it = r->windows.find({view, seq});
  return it != r->windows.end() && is_committed_local(r, view, it->second) ? 1 : 0;
}

int pbft_replica_get_stats(pbft_replica* r, pbft_replica_stats* out) {
  if (!r || !out) return PBFT_EINVAL;
  *out = r->stats;
  return PBFT_OK;
}

}  // extern "C"
