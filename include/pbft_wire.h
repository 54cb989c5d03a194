/*
 * pbft_wire.h — wire codec of the PBFT messages that feed the GPU verifier
 * (SURVEY.md §8f row 3).  Host C++ (pbft_amd/csrc/host/wire.cpp), compiled into
 * pbft_amd/libpbft_verify.so.
 *
 * Reference interfaces mirrored (ameya-deshmukh/pbft):
 *   pbft_uvi_encode / pbft_uvi_decode  unsigned-varint length prefix of the
 *       UviBytes framing (src/protocol_config.rs:51, :82 `UviBytes::default()`,
 *       unsigned-varint crate; max frame 128 MiB as its codec default)
 *   pbft_wire_encode_json              message_to_json src/protocol_config.rs:116-123
 *       = serde_json::to_string of the externally tagged `Message` enum
 *       (src/message.rs:7-31; structs :34-38, :105-115, :174-179, :214-219):
 *         {"Prepare":{"view":1,"sequence_number":2,"digest":"<128 hex>"}}
 *   pbft_wire_decode_json              bytes_to_message src/protocol_config.rs:125-129
 *       -> `impl From<Vec<u8>> for Message` (src/message.rs:15-19), which panics
 *       on bad input; here an error code is returned instead.
 *   pbft_wire_decode_votes             the ingress path PbftHandler ->
 *       message_to_handler_event (src/handler.rs:533-548): a byte stream of
 *       UviBytes frames straight into the verifier's struct-of-arrays batch.
 *
 * Signed-envelope extension (BASELINE north_star "a signed-message envelope in
 * message.rs"): PrePrepare / Prepare / Commit may carry two more fields after
 * the reference's ones, "replica" (u16 signer index = position in
 * network.json's "nodes") and "signature" (128 lowercase hex chars = R || S of
 * the Ed25519 signature over the 85-byte envelope of pbft_replica.h).  Messages
 * without them encode byte-identically to the reference.
 *
 * Binary record (zero-copy alternative to JSON, 160 bytes, 16-B aligned fields):
 *   [0,32) R  [32,64) S  [64,149) envelope  [149] pad  [150,152) key_idx LE
 *   [152,160) pad — consumed directly by pbft_verify_records_device.
 */
#ifndef PBFT_WIRE_H
#define PBFT_WIRE_H

#include <stddef.h>
#include <stdint.h>

#include "pbft_verify.h"

#ifdef __cplusplus
extern "C" {
#endif

#define PBFT_MSG_PREPREPARE 0
#define PBFT_MSG_PREPARE 1
#define PBFT_MSG_COMMIT 2
#define PBFT_MSG_CLIENT_REQUEST 3

#define PBFT_UVI_MAX_FRAME (128u * 1024u * 1024u)
#define PBFT_RECORD_BYTES 160

/* Frame decode status (pbft_wire_decode_votes) */
#define PBFT_WIRE_OK 0        /* signed PrePrepare/Prepare/Commit -> one SoA row */
#define PBFT_WIRE_EJSON 1     /* not a JSON Message of the reference schema */
#define PBFT_WIRE_EDIGEST 2   /* digest is not 128 hex chars               */
#define PBFT_WIRE_EUNSIGNED 3 /* no replica/signature fields               */
#define PBFT_WIRE_EKIND 4     /* ClientRequest (not signed by a replica)     */
#define PBFT_WIRE_ESIGNER 5   /* replica index >= n_replicas               */

typedef struct {
  uint32_t kind;     /* PBFT_MSG_* */
  uint64_t view;     /* PrePrepare / Prepare / Commit */
  uint64_t seq;      /* "sequence_number" */
  uint8_t digest[64];
  uint32_t digest_ok; /* 1: "digest" was 128 hex chars and is in digest[] */
  /* signed-envelope extension */
  uint32_t has_sig;
  uint32_t replica;
  uint8_t sig[64]; /* R || S */
  /* ClientRequest (standalone, or the PrePrepare's "message") */
  const char *operation; /* UTF-8, not NUL-terminated; decode: points into the arena */
  uint32_t operation_len;
  uint64_t timestamp;
  char client[64]; /* SocketAddr as serialized by serde ("127.0.0.1:8080"), NUL-terminated */
} pbft_wire_msg;

/* LEB128 unsigned varint.  encode: returns bytes written (1..10).
 * decode: 0 ok, 1 need more bytes, PBFT_EINVAL if overlong / non-minimal / > u64. */
size_t pbft_uvi_encode(uint64_t v, uint8_t out[10]);
int pbft_uvi_decode(const uint8_t *buf, size_t len, uint64_t *value, size_t *header_bytes);

/* serde_json encoding of m (compact, reference field order).  Writes at most cap
 * bytes, sets *len to the full length; returns 0, or PBFT_EINVAL if cap is too
 * small (nothing useful written) or the message is malformed. */
int pbft_wire_encode_json(const pbft_wire_msg *m, char *out, size_t cap, size_t *len);

/* One UviBytes frame (varint length + JSON) of m. Same conventions. */
int pbft_wire_encode_frame(const pbft_wire_msg *m, uint8_t *out, size_t cap, size_t *len);

/* Parse one JSON Message (any field order / whitespace, unknown fields ignored,
 * as serde does).  Unescaped strings go into arena (operation points there).
 * Returns 0 or PBFT_EINVAL. */
int pbft_wire_decode_json(const char *json, size_t len, pbft_wire_msg *out, char *arena, size_t arena_cap);

/* Decode a byte stream of UviBytes frames into the verifier's SoA batch.
 * Stops at the first incomplete frame, after max_rows signed votes, or after
 * max_frames frames.  For every decoded frame f: status[f] = PBFT_WIRE_*;
 * each OK frame appends row r: R[r], S[r], key_idx[r] = replica, msg[r] = the
 * 85-byte envelope (stride 85), kind[r] (0 PrePrepare, 1 Prepare, 2 Commit),
 * view[r], seq[r].  A PrePrepare row checks the primary's signature over the
 * CLAIMED digest only: the caller still recomputes the digest of its operation
 * (validate_digest, src/message.rs:139-145), as pbft_replica_push_frames does,
 * and checks that key_idx is the view's primary; key_idx of a vote must be the
 * authenticated connection's peer (src/behavior.rs:346, :380).  Outputs: *n_frames,
 * *n_rows, *consumed (bytes of whole frames).  Returns 0, or PBFT_EINVAL on a
 * framing error (bad varint / frame > PBFT_UVI_MAX_FRAME) at *consumed. */
int pbft_wire_decode_votes(const uint8_t *stream, size_t len, uint32_t n_replicas, uint64_t max_frames,
                           uint64_t max_rows, uint8_t *status, uint8_t *R, uint8_t *S, uint16_t *key_idx,
                           uint8_t *msg, uint8_t *kind, uint64_t *view, uint64_t *seq, uint64_t *n_frames,
                           uint64_t *n_rows, uint64_t *consumed);

/* N signed votes (kind[i] Prepare / Commit, view, seq, digest[64], replica, sig = R || S) as consecutive UviBytes
 * frames of their JSON Messages -- what a replica's connection carries when it multicasts its votes (the egress side
 * of pbft_replica_push_frames).  *len = the stream's full length; returns 0, or PBFT_EINVAL if cap is too small
 * (then *len still tells the length needed) or a kind is not a vote. */
int pbft_wire_encode_votes(uint64_t N, const uint8_t *kind, const uint64_t *view, const uint64_t *seq,
                           const uint8_t *digests, const uint32_t *replica, const uint8_t *sigs, uint8_t *out,
                           size_t cap, size_t *len);

/* Pack SoA rows into 160-byte binary records (layout above) and back. */
int pbft_records_pack(const uint8_t *R, const uint8_t *S, const uint16_t *key_idx, const uint8_t *msg,
                      uint32_t msg_stride, uint64_t N, uint8_t *records);

/* Verify N binary records resident on the device (zero-copy from the wire:
 * R, S, key index and envelope read in place with a 160-byte stride). */
int pbft_verify_records_device(pbft_ctx *ctx, const uint8_t *d_records, uint64_t N, uint64_t *d_bitmap,
                               void *stream);
/* Same from host records (one H2D copy of N x 160 bytes). Blocking. */
int pbft_verify_records(pbft_ctx *ctx, const uint8_t *records, uint64_t N, uint64_t *bitmap_out);

#ifdef __cplusplus
}
#endif
#endif /* PBFT_WIRE_H */
