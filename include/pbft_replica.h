/*
 * pbft_replica.h — C ABI of the host-side PBFT verification state machine that
 * feeds the GPU verifier: signed envelopes, a round
 * batcher keyed by (view, seq), the prepare / commit quorum predicates, a
 * watermark-bounded and garbage-collected log, and the libp2p PeerId -> key
 * binding.  Compiled into pbft_amd/libpbft_verify.so.
 *
 * Reference interfaces mirrored (ameya-deshmukh/pbft):
 *   pbft_replica_on_pre_prepare  Pbft::process_pre_prepare / validate_pre_prepare
 *                                src/behavior.rs:100-157 (digest check
 *                                src/message.rs:139-145, view check :134-141,
 *                                conflicting digest :144-151) plus the signature
 *                                check the reference leaves as a TODO (:127)
 *   pbft_replica_push            inject_node_event src/behavior.rs:340-412, but the
 *                                per-message validate_prepare / validate_commit
 *                                (:159-195) become "enqueue into the round window";
 *                                the signer is the AUTHENTICATED peer (the reference
 *                                keys votes by the connection's peer_id, :346, :380)
 *   pbft_replica_push_frames     PbftHandler -> message_to_handler_event
 *   pbft_replica_push_records    src/handler.rs:533-548 for one connection (UviBytes/
 *                                JSON frames, or 160-byte binary records)
 *   pbft_replica_flush_submit    the batched validation, non-blocking: every ready
 *   pbft_replica_flush_poll      sub-window's signatures in ONE GPU batch (votes
 *                                form, written into the verifier's pinned staging),
 *                                launched by _submit; _poll, called from the same
 *                                single-threaded loop as the reference's
 *                                NetworkBehaviour::poll (src/behavior.rs:416-426),
 *                                applies State::insert_prepare/insert_commit
 *                                (src/state.rs:49-67) for accepted ones only once
 *                                the bitmap is back.  pbft_replica_flush = both,
 *                                blocking.
 *   pbft_replica_prepared        Pbft::prepared src/behavior.rs:177-182 with the
 *                                paper's 2f threshold (reference: len >= 1, TODO)
 *   pbft_replica_committed_local Pbft::committed_local :214-223 with 2f+1 commits
 *                                keyed by (view, seq) (reference keys commits by
 *                                view only, src/state.rs:22-23)
 *   pbft_replica_set_log_window  the h / H watermarks the reference leaves as
 *   pbft_replica_stable_checkpoint  TODOs (src/behavior.rs:154, :192; its logs are
 *                                unbounded HashMaps, src/state.rs:9-11)
 *   pbft_key_from_peer_id        libp2p-core 0.31 PeerId of an Ed25519 identity
 *   pbft_replica_peer_index      (src/main.rs:39-40): 00 24 08 01 12 20 || A[32]
 *
 * Round batcher rules (one window per (view, seq), three sub-windows):
 *   - a signed PrePrepare is verified at the next flush (it gates the window);
 *   - the Prepare sub-window is READY once the distinct backups with an accepted
 *     or pending Prepare reach 2f (or all n-1 backups have sent one); the Commit
 *     sub-window once distinct replicas reach 2f+1 (or all n).  Each closes on
 *     its own count, so a phase-ordered run (Commits sent only after PREPARED)
 *     with f silent replicas progresses without a deadline flush;
 *   - flush(force = 1) (the caller's deadline) verifies everything pending;
 *   - at most one batch is in flight per replica; pushes during the flight are
 *     queued (a duplicate of an in-flight candidate is a duplicate) and go into
 *     the next batch;
 *   - a PrePrepare is taken only from the primary's own connection (frames and
 *     pbft_replica_on_pre_prepare alike: both take the authenticated peer);
 *   - events are decided as a batch is applied -- a window's as soon as its last
 *     rows in the batch are (a large batch comes back chunk by chunk), in
 *     (view, seq) order -- whether or not the caller's event buffer has room:
 *     undelivered events wait in the replica's queue for the next flush /
 *     flush_poll, and GC (the committed prefix, a stable checkpoint) never
 *     waits for delivery;
 *   - every candidate vote of a (kind, signer) is kept until one verifies (at
 *     most PBFT_MAX_CANDIDATES): a forged vote cannot pre-empt the real one
 *     (votes are keyed by the authenticated sender, so only the signer's own
 *     connection can fill its candidate slots);
 *     among accepted votes of one signer the last one wins (src/state.rs:56, :66);
 *   - seqs outside (h, h + log_window] are dropped; a window is erased once it
 *     is committed locally and every lower seq is too (h advances), or by
 *     pbft_replica_stable_checkpoint.
 *
 * Errors: negative PBFT_E* codes (pbft_verify.h); invalid signatures, wrong
 * digests, stale views and out-of-window seqs are dropped and counted, never
 * raised (the reference panics via .unwrap(), src/behavior.rs:97, :345, :371).
 */
#ifndef PBFT_REPLICA_H
#define PBFT_REPLICA_H

#include <stddef.h>
#include <stdint.h>

#include "pbft_verify.h"

#ifdef __cplusplus
extern "C" {
#endif

#define PBFT_KIND_PREPREPARE 0
#define PBFT_KIND_PREPARE 1
#define PBFT_KIND_COMMIT 2
#define PBFT_ENVELOPE_BYTES 85

#define PBFT_EVENT_PREPARED 1
#define PBFT_EVENT_COMMITTED_LOCAL 2
#define PBFT_EVENT_PRE_PREPARED 3 /* the PrePrepare's signature verified: send Prepare */

#define PBFT_MAX_CANDIDATES 4       /* pending votes kept per (window, kind, signer) */
#define PBFT_DEFAULT_LOG_WINDOW 4096 /* H - h */
#define PBFT_PEER_ID_BYTES 38       /* 00 24 08 01 12 20 || A[32] */

typedef struct pbft_replica pbft_replica;

typedef struct {
  uint64_t view, seq;
  uint32_t kind; /* PBFT_EVENT_* */
} pbft_round_event;

typedef struct {
  uint64_t pushed, verified, accepted, rejected_sig, rejected_digest, rejected_view, duplicates, batches;
  uint64_t rejected_watermark; /* seq outside (h, h + log_window]                      */
  uint64_t rejected_signer;    /* frame's "replica" is not the authenticated peer / not the primary */
  uint64_t dropped_flood;      /* candidates beyond PBFT_MAX_CANDIDATES                */
  uint64_t windows_gc;         /* windows erased (committed prefix or checkpoint)       */
  uint64_t low_watermark;      /* h                                                     */
  uint64_t live_windows;       /* windows currently held                                */
  uint64_t submit_ns;          /* host time inside pbft_replica_flush_submit (batch build + launch), summed */
  uint64_t apply_ns;           /* host time applying finished batches (bitmap -> votes, quorums, GC), summed */
} pbft_replica_stats;

/* Where the last push_many and the last flush spent their time (host clock, ns), so that a slow round can be
 * attributed from the record that shows it.  pbft_replica_get_timings copies them. */
typedef struct {
  uint64_t push_checks_ns;   /* the last pbft_replica_push_many: per-row checks (worker threads)                 */
  uint64_t push_windows_ns;  /*   the windows of its runs (serial, on the calling thread)                         */
  uint64_t push_rows_ns;     /*   the rows pushed (worker threads; with the early batch, its launches)            */
  uint64_t submit_segs_ns;   /* the last flush_submit that launched: the walk over the windows (segments)         */
  uint64_t submit_launch_ns; /*   the rest of it: adoption of an early batch, or the fill / copies / launches      */
  uint64_t wait_ns;          /* its batch: from the end of flush_submit to the flush_poll that found it complete  */
  uint64_t apply_partial_ns; /*   chunks applied by flush_poll while it ran                                       */
  uint64_t apply_final_ns;   /*   the rest applied once complete                                                  */
  uint64_t gc_ns;            /*   the evaluation of dirty windows and the GC after it                             */
  uint64_t polls;            /*   flush_poll calls that found it running                                          */
  uint64_t early_pieces;     /* single pushes before that flush_submit: early-batch pieces launched...            */
  uint64_t early_piece_ns;   /*   ...and the pushing thread's time inside those launches                          */
  uint64_t early_last_rows;  /* rows flush_submit launched as the early batch's last piece                        */
  /* the last push_many's worker spread (from the start of its pass): the first worker done with the checks, the
   * last worker to start pushing rows and the first one done -- a late start is a descheduled or slow-waking worker,
   * an early end far from push_rows_ns an imbalance or a worker interrupted mid-pass */
  uint64_t push_checks_end_min_ns;
  uint64_t push_rows_start_max_ns;
  uint64_t push_rows_end_min_ns;
} pbft_replica_timings;

/* Optional verifier override (tests without a GPU): same SoA contract as
 * pbft_verify_batch; returns 0 and fills bitmap_out. */
typedef int (*pbft_batch_verify_fn)(void *user, const uint8_t *R, const uint8_t *S, const uint16_t *key_idx,
                                    const uint8_t *msg, uint32_t msg_len, uint32_t msg_stride, uint64_t N,
                                    uint64_t *bitmap_out);

/* Optional asynchronous votes-form verifier (tests without a GPU, other backends): submit receives the
 * batch as columns -- sig[N][64] (R || S), key_idx[N], env_idx[N] and envelopes[n_env][85] (not the 72-byte
 * rows of pbft_verify_votes_stage); envelopes[env_idx[i]] is signature i's message; buffers owned by the replica, valid
 * until poll reports completion -- and returns 0 or a negative code; poll returns 1 once bitmap_out is
 * written, 0 while running, < 0 on failure. */
typedef int (*pbft_votes_submit_fn)(void *user, const uint8_t *sig, const uint16_t *key_idx, const uint32_t *env_idx,
                                    const uint8_t *envelopes, uint32_t n_env, uint64_t N, uint64_t *bitmap_out);
typedef int (*pbft_votes_poll_fn)(void *user);
/* (pbft_replica_set_verifier / _set_votes_verifier: the last one installed serves the flushes; NULL
 * uninstalls, and with neither the replica uses its GPU context.) */

/* Optional request-digest override (tests without a GPU): Blake2b-512 of op. */
typedef int (*pbft_digest_fn)(void *user, const uint8_t *op, uint32_t op_len, uint8_t digest_out[64]);

/* n replicas (f = (n-1)/3), this replica's id, the replica key set keys[n][32]
 * (also installed on ctx with pbft_verify_set_keys).  ctx may be NULL only if a
 * verifier override is installed before the first flush.  The primary of view v
 * is replica v mod n (Castro-Liskov p = v mod |R|). */
int pbft_replica_create(pbft_ctx *ctx, uint32_t n, uint32_t self_id, const uint8_t *keys, pbft_replica **out);
/* The same replica over several verifier contexts (one per GPU of the node, or clones of one GPU's context; distinct,
 * each with the replica key set installed; ctxs[0] also serves digests and small batches).  A flush of >= 2^16 rows
 * is cut into one contiguous slice per context (balanced by rows, at window-phase boundaries, each slice 64-row
 * aligned); every context stages its slice and the envelope table in its own pinned staging and launches it chunk
 * by chunk as the worker threads fill it, so the slices' host-to-device copies run on every GPU's PCIe link at once
 * (one replica used one GPU and one link of eight); flush_poll applies rows as each context's bitmap
 * words land, in row order.  n_ctx <= PBFT_MAX_REPLICA_CTX.  pbft_replica_update_keys updates every context. */
#define PBFT_MAX_REPLICA_CTX 16
int pbft_replica_create_multi(pbft_ctx *const *ctxs, uint32_t n_ctx, uint32_t n, uint32_t self_id,
                              const uint8_t *keys, pbft_replica **out);
/* Replica idx[i] (< n, distinct) gets the key A[i][32] -- a peer admitted after start-up (Pbft::add_peer,
 * src/behavior.rs:45-61, fed by mDNS discovery src/network_behaviour_composer.rs:24-33): its PeerId now maps to
 * replica idx[i] (pbft_replica_peer_index) and, with a GPU context, only its comb tables are rebuilt
 * (pbft_verify_update_keys; key_ok as there).  Votes already accepted under the old key stay; candidates still
 * pending are verified under the new key.  PBFT_EBUSY while a batch is in flight.  PBFT_EINVAL if two new keys
 * are equal or a new key is held by a slot that is not being replaced (one of the two would be unreachable by
 * PeerId).  The GPU key set belongs to the context (and its clones): a context serves ONE replica -- another
 * replica on it would verify against the new key while its PeerId map keeps the old one. */
int pbft_replica_update_keys(pbft_replica *r, const uint32_t *idx, const uint8_t *A, uint32_t m, uint8_t *key_ok);
int pbft_replica_destroy(pbft_replica *r);
int pbft_replica_set_verifier(pbft_replica *r, pbft_batch_verify_fn fn, void *user);
int pbft_replica_set_votes_verifier(pbft_replica *r, pbft_votes_submit_fn submit, pbft_votes_poll_fn poll,
                                    void *user);
int pbft_replica_set_digest_fn(pbft_replica *r, pbft_digest_fn fn, void *user);
/* H - h (default PBFT_DEFAULT_LOG_WINDOW; >= 1). */
int pbft_replica_set_log_window(pbft_replica *r, uint64_t log_window);

/* Encode the 85-byte signed envelope "PBFT" || kind || view LE || seq LE || digest. */
void pbft_envelope(uint8_t out[PBFT_ENVELOPE_BYTES], uint8_t kind, uint64_t view, uint64_t seq,
                   const uint8_t digest[64]);

/* A PrePrepare for (view, seq) carrying the client operation bytes and the
 * primary's signature (R || S over the kind-0 envelope of the claimed digest),
 * received from replica `peer_idx` -- the AUTHENTICATED sender (the connection's
 * peer, pbft_replica_peer_index; inject_node_event's peer_id, src/behavior.rs:304,
 * PrePrepare arm :310-318), never a field of the message.  Unless peer_idx is the
 * view's primary the PrePrepare is dropped before any work (counted in
 * rejected_signer): a backup relaying junk PrePrepares cannot fill the window's
 * PBFT_MAX_CANDIDATES slots ahead of the primary's real one.  Recomputes the
 * Blake2b-512 digest (GPU, or the digest override); returns 1 if queued for
 * signature verification (PBFT_EVENT_PRE_PREPARED at the flush that accepts it),
 * 0 if dropped (not from the primary / digest mismatch / wrong view / out of
 * window / conflicting digest already accepted for (view, seq)).  digest_out
 * (optional) receives the recomputed digest (left untouched when the sender is
 * rejected). */
int pbft_replica_on_pre_prepare(pbft_replica *r, uint32_t peer_idx, uint64_t view, uint64_t seq, const uint8_t *op,
                                uint32_t op_len, const uint8_t claimed_digest[64], const uint8_t primary_sig[64],
                                uint8_t digest_out[64]);

/* A signed Prepare/Commit from replica `signer` (sig = R || S).  `signer` must be
 * the AUTHENTICATED sender (the connection's peer, pbft_replica_peer_index),
 * never a field of the message.  Returns 1 queued, 0 dropped. */
int pbft_replica_push(pbft_replica *r, uint8_t kind, uint64_t view, uint64_t seq, const uint8_t digest[64],
                      uint32_t signer, const uint8_t sig[64]);

/* N pushes in one call (kind[i], view[i], seq[i], digests[i][64], signer[i], sigs[i][64]); *queued = how many
 * were queued.  Returns 0 or the first negative code.
 * Every queued vote's 72-byte staged row (PBFT_VOTES_ROW_BYTES) goes into the replica's pinned row arena as it is
 * pushed (r05), by tasks of consecutive windows that the worker threads take as they free up (r06).  With GPU
 * contexts, no override verifier, no batch in flight and >= 2^17 rows, push_many also starts verifying the arena
 * while it pushes ("early batch": pieces of 2^17 rows launched through pbft_verify_votes_open / _piece / _close as
 * soon as the tasks below their ends are done, each context taking a contiguous run of tasks); the next flush_submit
 * adopts that batch when the arena is unchanged since (and flush_poll applies its windows as its pieces land), and
 * otherwise finishes it and verifies the arena again -- so the contexts are busy between push_many and the flush,
 * and a key update or a verifier change in between waits for the early batch first.  Environment (read per call,
 * for A/B runs): PBFT_REPLICA_EARLY=0 (no early batch), PBFT_MANY_PIECE (rows per piece, default 2^17),
 * PBFT_PUSH_TASKS (tasks per thread, default 8), PBFT_ADOPT_PARTIAL=0 (an adopted batch applied once, when done),
 * PBFT_REPLICA_DIRECT=0 (flush_submit fills the context's staging instead of handing the arena over),
 * PBFT_APPLY_PREFETCH (segments ahead, 0 = off, default 1), PBFT_REPLICA_THREADS (worker threads, default 16),
 * PBFT_NUMA_BIND=0 (the workers are kept on the NUMA node of `digests` by default); read once: PBFT_STREAM_STORES=0
 * (plain stores for the rows). */
int pbft_replica_push_many(pbft_replica *r, uint64_t N, const uint8_t *kind, const uint64_t *view, const uint64_t *seq,
                           const uint8_t *digests, const uint32_t *signer, const uint8_t *sigs, uint64_t *queued);

/* Ingress straight from one connection's byte stream (include/pbft_wire.h):
 * decode UviBytes frames (src/protocol_config.rs:49-69 upgrade_inbound); signed
 * Prepare / Commit frames whose "replica" equals peer_idx (the authenticated
 * connection) are pushed, signed PrePrepare frames go to on_pre_prepare (their
 * signature must be the view's primary's), everything else is counted in
 * *dropped.  *consumed = bytes of whole frames (keep the rest for the next
 * read).  Returns 0, or PBFT_EINVAL on a framing error. */
int pbft_replica_push_frames(pbft_replica *r, uint32_t peer_idx, const uint8_t *stream, size_t len,
                             uint64_t *consumed, uint64_t *pushed, uint64_t *dropped);
/* The same from one connection's stream of 160-byte binary records (PBFT_RECORD_BYTES, include/pbft_wire.h:
 * R || S, the 85-byte signed envelope, the signer's key index LE at byte 150), the zero-copy alternative to JSON
 * frames: Prepare / Commit records whose key index equals peer_idx are pushed, others counted
 * in *dropped (a record whose key index is not the connection's peer also in rejected_signer; PrePrepares need
 * their operation bytes: on_pre_prepare or a JSON frame).  *consumed = bytes of whole records.  Returns 0 or the
 * first negative code of a push (then *consumed stops before that record). */
int pbft_replica_push_records(pbft_replica *r, uint32_t peer_idx, const uint8_t *stream, size_t len,
                              uint64_t *consumed, uint64_t *pushed, uint64_t *dropped);

/* Non-blocking flush.  _submit: collect every READY sub-window (force = every pending candidate) into one
 * batch and launch it; *n_rows = its signatures (0: nothing launched); PBFT_EBUSY while a batch is in flight.
 * _poll: 1 once no batch is in flight -- the finished batch's accepted votes inserted, the events it
 * decided queued, the committed prefix garbage-collected, and up to max_events queued events written to
 * events (*n_events; the rest stay queued for the next call); 0 while the GPU is still working (nothing
 * written); < 0 if the batch failed (its candidates are pending again).  Call _poll from the event loop
 * (the reference's NetworkBehaviour::poll, src/behavior.rs:416-426). */
int pbft_replica_flush_submit(pbft_replica *r, int force, uint64_t *n_rows);
int pbft_replica_flush_poll(pbft_replica *r, pbft_round_event *events, uint32_t max_events, uint32_t *n_events);
/* 1 while a batch is in flight, else 0. */
int pbft_replica_in_flight(pbft_replica *r);

/* Blocking flush: completes a batch still in flight (its events are queued), then _submit + wait + _poll. */
int pbft_replica_flush(pbft_replica *r, int force, pbft_round_event *events, uint32_t max_events,
                       uint32_t *n_events);

/* Stable checkpoint at seq (PBFT §4.3): h = max(h, seq); windows <= h erased. */
int pbft_replica_stable_checkpoint(pbft_replica *r, uint64_t seq);

/* Quorum predicates.  A garbage-collected seq reports 1 only if this replica committed it locally (a
 * stable checkpoint raises h without deciding anything here). */
int pbft_replica_prepared(pbft_replica *r, uint64_t view, uint64_t seq);
int pbft_replica_committed_local(pbft_replica *r, uint64_t view, uint64_t seq);
int pbft_replica_get_stats(pbft_replica *r, pbft_replica_stats *out);
int pbft_replica_get_timings(pbft_replica *r, pbft_replica_timings *out);

/* libp2p PeerId <-> Ed25519 key.  A PeerId of an Ed25519 identity is the
 * identity multihash of the protobuf-encoded public key: 00 24 08 01 12 20 || A.
 * pbft_key_from_peer_id: 0 and A[32], or PBFT_EINVAL (wrong length / prefix).
 * pbft_peer_id_from_key: writes the 38 bytes.
 * pbft_key_from_peer_id_b58: the same from the base58btc text form ("12D3KooW...").
 * pbft_replica_peer_index: the replica index whose key the PeerId carries, or
 * PBFT_EINVAL if it is malformed or not a replica of this set. */
int pbft_key_from_peer_id(const uint8_t *peer_id, size_t len, uint8_t A[32]);
void pbft_peer_id_from_key(const uint8_t A[32], uint8_t peer_id[PBFT_PEER_ID_BYTES]);
int pbft_key_from_peer_id_b58(const char *text, size_t len, uint8_t A[32]);
int pbft_replica_peer_index(pbft_replica *r, const uint8_t *peer_id, size_t len);

#ifdef __cplusplus
}
#endif
#endif /* PBFT_REPLICA_H */
