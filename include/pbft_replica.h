/*
 * pbft_replica.h — C ABI of the host-side PBFT verification state machine that
 * feeds the GPU verifier: signed envelopes, a round
 * batcher keyed by (view, seq), and the prepare / commit quorum predicates.
 * Compiled into pbft_amd/libpbft_verify.so.
 *
 * Reference interfaces mirrored (ameya-deshmukh/pbft):
 *   pbft_replica_on_pre_prepare  Pbft::process_pre_prepare / validate_pre_prepare
 *                                src/behavior.rs:100-157 (digest check
 *                                src/message.rs:139-145, view check :134-141,
 *                                conflicting digest :144-151)
 *   pbft_replica_push            PbftHandler message_to_handler_event
 *                                src/handler.rs:533-548 -> inject_node_event
 *                                src/behavior.rs:340-412, but the per-message
 *                                validate_prepare/validate_commit (:159-195) become
 *                                "enqueue into the round window"
 *   pbft_replica_flush           the batched validation: every closed window's
 *                                Prepare+Commit signatures in ONE GPU batch, then
 *                                State::insert_prepare/insert_commit
 *                                (src/state.rs:49-67) for accepted ones only
 *   pbft_replica_prepared        Pbft::prepared src/behavior.rs:177-182 with the
 *                                paper's 2f threshold (reference: len >= 1, TODO)
 *   pbft_replica_committed_local Pbft::committed_local :214-223 with 2f+1 commits
 *                                keyed by (view, seq) (reference keys commits by
 *                                view only, src/state.rs:22-23)
 *
 * Errors: negative PBFT_E* codes (pbft_verify.h); invalid signatures, wrong
 * digests and stale views are dropped and counted, never raised (the reference
 * panics via .unwrap(), src/behavior.rs:97, :345, :371).
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

typedef struct pbft_replica pbft_replica;

typedef struct {
  uint64_t view, seq;
  uint32_t kind; /* PBFT_EVENT_* */
} pbft_round_event;

typedef struct {
  uint64_t pushed, verified, accepted, rejected_sig, rejected_digest, rejected_view, duplicates, batches;
} pbft_replica_stats;

/* Optional verifier override (tests without a GPU): same SoA contract as
 * pbft_verify_batch; returns 0 and fills bitmap_out. */
typedef int (*pbft_batch_verify_fn)(void *user, const uint8_t *R, const uint8_t *S, const uint16_t *key_idx,
                                    const uint8_t *msg, uint32_t msg_len, uint32_t msg_stride, uint64_t N,
                                    uint64_t *bitmap_out);

/* Optional request-digest override (tests without a GPU): Blake2b-512 of op. */
typedef int (*pbft_digest_fn)(void *user, const uint8_t *op, uint32_t op_len, uint8_t digest_out[64]);

/* n replicas (f = (n-1)/3), this replica's id, the replica key set keys[n][32]
 * (also installed on ctx with pbft_verify_set_keys).  ctx may be NULL only if a
 * verifier override is installed before the first flush. */
int pbft_replica_create(pbft_ctx *ctx, uint32_t n, uint32_t self_id, const uint8_t *keys, pbft_replica **out);
int pbft_replica_destroy(pbft_replica *r);
int pbft_replica_set_verifier(pbft_replica *r, pbft_batch_verify_fn fn, void *user);
int pbft_replica_set_digest_fn(pbft_replica *r, pbft_digest_fn fn, void *user);

/* Encode the 85-byte signed envelope "PBFT" || kind || view LE || seq LE || digest. */
void pbft_envelope(uint8_t out[PBFT_ENVELOPE_BYTES], uint8_t kind, uint64_t view, uint64_t seq,
                   const uint8_t digest[64]);

/* Accept a PrePrepare for (view, seq) carrying the client operation bytes.
 * Recomputes the Blake2b-512 digest on the GPU; returns 1 accepted, 0 dropped
 * (digest mismatch / wrong view / conflicting digest for (view, seq)).
 * digest_out (optional) receives the digest. */
int pbft_replica_on_pre_prepare(pbft_replica *r, uint64_t view, uint64_t seq, const uint8_t *op, uint32_t op_len,
                                const uint8_t claimed_digest[64], uint8_t digest_out[64]);

/* Ingress of a signed Prepare/Commit from replica `signer` (sig = R || S). */
int pbft_replica_push(pbft_replica *r, uint8_t kind, uint64_t view, uint64_t seq, const uint8_t digest[64],
                      uint32_t signer, const uint8_t sig[64]);

/* Ingress straight from the wire (include/pbft_wire.h): decode a byte stream of
 * UviBytes frames (src/protocol_config.rs:50-76 upgrade_inbound) and push every
 * signed Prepare / Commit into its round window; other frames are counted in
 * *dropped.  *consumed = bytes of whole frames (keep the rest for the next read).
 * Returns 0, or PBFT_EINVAL on a framing error. */
int pbft_replica_push_frames(pbft_replica *r, const uint8_t *stream, size_t len, uint64_t *consumed,
                             uint64_t *pushed, uint64_t *dropped);

/* Verify every closed round window in one batch (force = also open windows),
 * insert the accepted votes and report newly reached quorums. */
int pbft_replica_flush(pbft_replica *r, int force, pbft_round_event *events, uint32_t max_events,
                       uint32_t *n_events);

int pbft_replica_prepared(pbft_replica *r, uint64_t view, uint64_t seq);
int pbft_replica_committed_local(pbft_replica *r, uint64_t view, uint64_t seq);
int pbft_replica_get_stats(pbft_replica *r, pbft_replica_stats *out);

#ifdef __cplusplus
}
#endif
#endif /* PBFT_REPLICA_H */
