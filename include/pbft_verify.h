/*
 * pbft_verify.h — C ABI of the MI355X batch Ed25519 verifier that gates PBFT's
 * prepare/commit quorums.  Shared library: pbft_amd/libpbft_verify.so (gfx950).
 *
 * Reference interfaces each entry point replaces (ameya-deshmukh/pbft):
 *   pbft_verify_batch*     validate_prepare  src/behavior.rs:159-175 and
 *                          validate_commit   src/behavior.rs:184-195, whose
 *                          signature checks are TODOs (src/behavior.rs:127, :185);
 *                          called per message from inject_node_event
 *                          src/behavior.rs:340-412.  Here one call verifies a
 *                          whole (view, seq) round window and returns a bitmap.
 *   pbft_verify_set_keys   libp2p-core 0.31 identity::ed25519 PublicKey decode
 *                          (keys created at src/main.rs:39-40; PeerId bytes are
 *                          00 24 08 01 12 20 || A[32]).
 *   pbft_digest_blake2b512 digest() src/message.rs:209-212 (request digest,
 *                          checked by PrePrepare::validate_digest :139-145).
 *   pbft_digest_sha256     the SHA-256 request digest named by BASELINE.json.
 *   pbft_sign_batch        RFC 8032 signing of the replicas' own Prepare/Commit
 *                          envelopes (the reference multicasts them unsigned,
 *                          src/behavior.rs:116-122, :356-362).
 *
 * Semantics: ed25519-dalek 1.0.1 PublicKey::verify_strict (Cargo.lock:668-679):
 * s < L, A and R decompress per curve25519-dalek 3.2.1, neither small order,
 * k = SHA-512(R || A || M) mod L over the raw bytes, accept iff
 * [s]B - [k]A == R as points.  An invalid signature is NOT an error: bit = 0.
 *
 * Conventions:
 *  - Return 0 on success, a negative PBFT_E* code on failure; never aborts.
 *  - Caller owns host buffers; the context owns its device buffers.
 *  - Bitmaps: bit i is bit (i % 64) of word i / 64 (LSB first); bits >= N are 0.
 *  - One context per host thread (contexts are not internally locked).
 *  - Byte strings (R, S, A, keys) are the 32-byte little-endian encodings.
 */
#ifndef PBFT_VERIFY_H
#define PBFT_VERIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PBFT_OK 0
#define PBFT_EINVAL (-1)   /* bad argument (null pointer, size out of range)   */
#define PBFT_EHIP (-2)     /* HIP runtime error (message in pbft_last_error)   */
#define PBFT_ENOKEYS (-3)  /* pbft_verify_set_keys has not been called        */
#define PBFT_ENOMEM (-4)   /* device or pinned allocation failed              */
#define PBFT_ENODEV (-5)   /* no gfx950 device at the requested ordinal       */
#define PBFT_EBUSY (-6)    /* an async batch is in flight on this context     */

typedef struct pbft_ctx pbft_ctx;

/* Create a context on HIP device `device`; builds the base-point comb table. */
int pbft_verify_ctx_create(int device, pbft_ctx **out);
int pbft_verify_ctx_destroy(pbft_ctx *ctx);

/* Install the replica key set A[n][32] (n <= 65535).  Decompresses every key,
 * rejects small-order keys, and builds each key's -A comb table in HBM.
 * key_ok (optional, n bytes): 1 = key usable, 0 = every signature under it
 * rejects (bad encoding or small order).  Replaces any previous key set.
 * A re-key whose tables fit the current set's allocation (at most as many
 * keys, same or smaller comb plan) reuses that allocation (tables rebuilt in
 * place; no HBM freed or allocated: freed VRAM is wiped by the driver before it
 * can be handed out again, seconds for a key set) unless a clone shares the
 * set; otherwise the old tables are freed first.  The context is busy
 * (blocking call) throughout. */
int pbft_verify_set_keys(pbft_ctx *ctx, const uint8_t *A, uint32_t n, uint8_t *key_ok);

/* Replace m keys of the installed set: key idx[i] (< n, distinct) becomes
 * A[i][32]; only those m keys' tables are rebuilt (the reference admits peers
 * one at a time: Pbft::add_peer src/behavior.rs:45-61, fed by mDNS discovery
 * src/network_behaviour_composer.rs:24-33 -- a replica slot can be installed
 * with a placeholder key, key_ok 0, and filled here when its peer appears).
 * key_ok (optional, m bytes) as for set_keys.  The set is updated in place for
 * every context sharing it (pbft_verify_ctx_clone): no batch may be in flight
 * on any of them (the call synchronises the device first).  On failure: if
 * nothing was written yet (scratch allocation, key upload) the set is
 * unchanged; otherwise the m slots' key_ok is cleared in the shared set (every
 * context holding it rejects signatures under them; the other keys work). */
int pbft_verify_update_keys(pbft_ctx *ctx, const uint32_t *idx, const uint8_t *A, uint32_t m, uint8_t *key_ok);
/* Slots idx[0..m) of the installed set reject every signature from now on (key_ok cleared in the shared set; the
 * tables stay) until a later set_keys / update_keys installs them again -- a replica whose key update failed on
 * one of its contexts revokes the slots on all of them (pbft_replica_update_keys).  Synchronises the device. */
int pbft_verify_revoke_keys(pbft_ctx *ctx, const uint32_t *idx, uint32_t m);
/* *id = an identity of the key set the context verifies against, equal for contexts sharing one
 * (pbft_verify_ctx_clone); 0 without a key set. */
int pbft_verify_key_set_id(pbft_ctx *ctx, uint64_t *id);

/* Phases of the last pbft_verify_set_keys / pbft_verify_update_keys on this
 * context (host wall time, ms). */
typedef struct {
  double total_ms;
  double meminfo_ms;     /* hipMemGetInfo (plan selection)                         */
  double free_ms;        /* releasing the previous key tables (hipFree)            */
  double alloc_ms;       /* allocating the new ones (hipMalloc)                    */
  double build_ms;       /* key upload + decompression + comb-table kernels + sync */
  uint32_t keys_built;   /* keys whose tables were (re)built                       */
  uint32_t reused;       /* 1: the existing table allocation was kept              */
  uint64_t table_bytes;  /* HBM held by the key tables                             */
} pbft_key_stats;
int pbft_verify_key_stats(pbft_ctx *ctx, pbft_key_stats *out);

/* A second context on the same device that shares the parent's base-point
 * table and its CURRENT key set (reference-counted; a later set_keys on either
 * context replaces only that context's key set), with its own HIP stream,
 * staging and workspace: one context per host thread / in-flight stream for
 * pipelined serving of small batches (BASELINE config #5).  The clone starts
 * with the parent's tuning options (pbft_verify_set_option). */
int pbft_verify_ctx_clone(pbft_ctx *parent, pbft_ctx **out);

/* Blocking batch verify from host buffers (PCIe copies included).
 * R[N][32], S[N][32], key_idx[N] (index into the key set), msg[N][msg_stride]
 * of which the first msg_len bytes are the signed message.  bitmap_out has
 * ceil(N/64) words. */
int pbft_verify_batch(pbft_ctx *ctx, const uint8_t *R, const uint8_t *S, const uint16_t *key_idx,
                      const uint8_t *msg, uint32_t msg_len, uint32_t msg_stride, uint64_t N,
                      uint64_t *bitmap_out);

/* The same batch sharded over n_ctx distinct contexts (several GPUs of this
 * process and/or cloned contexts of one GPU): contiguous 64-aligned shards,
 * launched concurrently, bitmap words written in place.  Blocking.  (One
 * process per GPU with an RCCL all-gather is the other layout: bench.py.) */
int pbft_verify_batch_multi(pbft_ctx *const *ctxs, uint32_t n_ctx, const uint8_t *R, const uint8_t *S,
                            const uint16_t *key_idx, const uint8_t *msg, uint32_t msg_len, uint32_t msg_stride,
                            uint64_t N, uint64_t *bitmap_out);

/* Single-process multi-GPU round with the bitmap exchange on RCCL (SURVEY.md §8b "Conventions", §8e):
 * pbft_multi_create takes one context per device (distinct devices, in rank order) and builds an RCCL
 * communicator over them (ncclCommInitAll; RCCL is loaded at run time: librccl.so.1, the library torch and
 * /opt/rocm ship).  pbft_verify_batch_device_multi: rank r verifies its shard -- n[r] signatures whose
 * device-resident columns d_R[r], d_S[r], d_key_idx[r], d_msg[r] live on ctx r's device (the layout of
 * pbft_verify_batch_device) -- into words [r * words_per_rank, r * words_per_rank + ceil(n[r] / 64)) of
 * d_bitmap[r], then one ncclAllGather (in place, ncclUint64, words_per_rank words per rank) leaves every
 * rank's d_bitmap[r] holding all n_ctx * words_per_rank words (rank-major, each rank's slice padded with
 * zero words to words_per_rank >= ceil(n[r] / 64)).  Enqueued on each context's stream; pbft_multi_sync
 * waits for all ranks.  (One process per GPU with torch.distributed is the other layout: bench.py.) */
typedef struct pbft_multi pbft_multi;
int pbft_multi_create(pbft_ctx *const *ctxs, uint32_t n_ctx, pbft_multi **out);
int pbft_multi_destroy(pbft_multi *m);
int pbft_verify_batch_device_multi(pbft_multi *m, const uint8_t *const *d_R, const uint8_t *const *d_S,
                                   const uint16_t *const *d_key_idx, const uint8_t *const *d_msg, uint32_t msg_len,
                                   uint32_t msg_stride, const uint64_t *n, uint64_t words_per_rank,
                                   uint64_t *const *d_bitmap);
int pbft_multi_sync(pbft_multi *m);

/* Non-blocking form: enqueue copies + kernel, return; pbft_verify_poll / pbft_verify_wait complete it
 * (bitmap_out is written by the call that observes completion).  One batch in flight per context.
 * Host buffers in pinned memory (hipHostMalloc / hipHostRegister) are DMA'd in place and must stay valid
 * until completion; pageable buffers are first copied into the context's pinned staging (a CPU memcpy,
 * then asynchronous DMA), so they may be reused as soon as the call returns.  Replaces the blocking
 * validate_prepare / validate_commit call inside inject_node_event (src/behavior.rs:345, :371) with a
 * submit from, and a poll in, the swarm's single-threaded poll loop (src/behavior.rs:416-426). */
int pbft_verify_batch_async(pbft_ctx *ctx, const uint8_t *R, const uint8_t *S, const uint16_t *key_idx,
                            const uint8_t *msg, uint32_t msg_len, uint32_t msg_stride, uint64_t N,
                            uint64_t *bitmap_out);
/* Returns 1 if the in-flight batch finished (bitmap written; also 1 when nothing is in flight), 0 if still
 * running, < 0 on error (the batch is then dropped). */
int pbft_verify_poll(pbft_ctx *ctx);
int pbft_verify_wait(pbft_ctx *ctx);

/* Votes form, non-blocking (see pbft_verify_votes below for the layout): same buffer rules as
 * pbft_verify_batch_async; complete with pbft_verify_poll / pbft_verify_wait. */
int pbft_verify_votes_async(pbft_ctx *ctx, const uint8_t *R, const uint8_t *S, const uint16_t *key_idx,
                            const uint32_t *env_idx, const uint8_t *envelopes, uint32_t n_env, uint64_t N,
                            uint64_t *bitmap_out);
/* Staged votes form: pbft_verify_votes_stage returns the context's pinned host staging for a batch of N
 * signatures over n_env envelopes, laid out as N rows of PBFT_VOTES_ROW_BYTES (72) bytes -- the 64-byte
 * signature R || S as it travels, key_idx (u16) at byte 64, two zero bytes, env_idx (u32) at byte 68 -- then
 * envelopes[n_env][85].  sig, key_idx and env_idx point at row 0's fields (row i's at + i * row_stride bytes), so
 * one DMA per chunk moves everything a chunk's kernels read (three per chunk with separate columns: the two
 * small copies and their gaps cost 23 % of the copy engine's time, profiles/r04/votes_copies.txt).  Valid until the
 * next call on this context that uses the staging (another stage, or any host-buffer submit: pageable inputs are
 * copied there, and a bigger batch reallocates it; such a call also voids the stage, so a later
 * pbft_verify_votes_submit fails with PBFT_EINVAL) -- the caller fills it in place and pbft_verify_votes_submit
 * launches it asynchronously.  This is what pbft_replica_flush_submit uses. */
#define PBFT_VOTES_ROW_BYTES 72
#define PBFT_VOTES_ROW_KEY 64
#define PBFT_VOTES_ROW_ENV 68
typedef struct {
  uint8_t *sig;        /* row i: sig + i * row_stride, 64 bytes */
  uint16_t *key_idx;   /* row i: (uint8_t *)key_idx + i * row_stride */
  uint32_t *env_idx;   /* row i: (uint8_t *)env_idx + i * row_stride */
  uint8_t *envelopes;  /* [n_env][85], contiguous */
  uint32_t row_stride; /* PBFT_VOTES_ROW_BYTES */
} pbft_votes_staging;
int pbft_verify_votes_stage(pbft_ctx *ctx, uint64_t N, uint32_t n_env, pbft_votes_staging *out);
int pbft_verify_votes_submit(pbft_ctx *ctx, uint64_t N, uint32_t n_env, uint64_t *bitmap_out);
/* Progressive form of pbft_verify_votes_submit, so that filling the staging, the GPU and applying the results
 * overlap: after pbft_verify_votes_stage and with the envelopes filled, _submit_begin launches the envelope
 * table; the caller then fills the signature rows front to back and calls _submit_rows(rows) whenever rows
 * [0, rows) are filled -- every whole chunk of the schedule below inside is copied and launched -- and finally
 * _submit_rows(N).  pbft_verify_poll_rows returns like pbft_verify_poll and sets *rows_done: the bitmap words of
 * rows [0, rows_done) are already in bitmap_out (each chunk's words come back as soon as its kernels finish).
 * pbft_replica_flush_submit / _flush_poll use this.  Until _submit_rows(N) pbft_verify_poll reports "running"
 * and pbft_verify_wait fails with PBFT_EBUSY; a failing _submit_rows drops the batch. */
int pbft_verify_votes_submit_begin(pbft_ctx *ctx, uint64_t N, uint32_t n_env, uint64_t *bitmap_out);
/* Chunk schedule of the votes forms from host buffers (each chunk: its H2D on the copy stream, its kernels, and in
 * the progressive form its bitmap words back): a batch of at most PBFT_VOTES_CHUNK_ROWS rows is one chunk; a larger
 * one starts with a PBFT_VOTES_FIRST_ROWS-row chunk and a 2 x PBFT_VOTES_FIRST_ROWS-row one, so that the first copy
 * starts after a small part of the rows is filled, then PBFT_VOTES_CHUNK_ROWS-row chunks, and it ends with a
 * ~2 x PBFT_VOTES_FIRST_ROWS-row and a ~PBFT_VOTES_FIRST_ROWS-row chunk, so that little compute is left once the
 * last copy lands (the copies are the bound; r04: profiles/r04/votes_copies.txt).  Every chunk but the last is a
 * multiple of 64 rows.  The chunk starting at row lo of an n-row batch ends at PBFT_VOTES_CHUNK_END(lo, n). */
#define PBFT_VOTES_CHUNK_ROWS (1u << 18)
#define PBFT_VOTES_FIRST_ROWS (1u << 16)
static inline uint64_t pbft_votes_chunk_end(uint64_t lo, uint64_t n) {
  const uint64_t F = PBFT_VOTES_FIRST_ROWS, C = PBFT_VOTES_CHUNK_ROWS, r = n - lo;
  if (n <= C || lo >= n) return n;
  if (lo == 0) return F;
  if (lo == F) return 3 * F < n ? 3 * F : n;
  if (r > C + 3 * F) return lo + C;                      /* at least 3F rows stay */
  if (r > 4 * F) return lo + ((r - 3 * F) & ~(uint64_t)63); /* 2F + F stay */
  if (r > 2 * F) return lo + ((r - F) & ~(uint64_t)63);     /* F stays */
  return n;
}
#define PBFT_VOTES_CHUNK_END(lo, n) pbft_votes_chunk_end((uint64_t)(lo), (uint64_t)(n))
int pbft_verify_votes_submit_rows(pbft_ctx *ctx, uint64_t rows);
int pbft_verify_poll_rows(pbft_ctx *ctx, uint64_t *rows_done);
/* Votes rows the caller already holds in pinned host memory (pbft_host_alloc): rows[N] of PBFT_VOTES_ROW_BYTES laid
 * out as pbft_verify_votes_stage describes, then envelopes[n_env][85] in a buffer of its own (+ 16 readable bytes);
 * both stay unchanged until the batch completes.  Launches the whole batch at once on the chunk schedule above, each
 * chunk's H2D straight from the caller's rows (no staging, no fill), and completes like the progressive form
 * (pbft_verify_poll_rows / pbft_verify_wait).  pbft_replica writes every vote's row into such a buffer when the vote
 * is pushed, so its flush touches no vote a second time. */
int pbft_verify_votes_submit_host(pbft_ctx *ctx, const uint8_t *rows, uint64_t N, const uint8_t *envelopes,
                                  uint32_t n_env, uint64_t *bitmap_out);
/* A votes batch in pieces, for rows that are still being written while the first ones are verified
 * (pbft_replica_push_many launches each part of the replica's row arena as its worker threads finish it):
 * _open(n_cap, env_cap, bitmap_out) starts a batch of at most n_cap rows over at most env_cap envelopes; each
 * _piece(rows, row_lo, row_hi, envelopes, env_lo, env_hi) copies envelopes [env_lo, env_hi) (their block-2
 * schedules computed on the GPU) and launches rows [row_lo, row_hi) -- rows and envelopes addressed from the same
 * base pointers in every call, pinned (pbft_host_alloc), unchanged until the batch completes; pieces in order and
 * contiguous (row_lo = the previous row_hi, a multiple of 64; env_lo = the previous env_hi), a row may name any
 * envelope below its piece's env_hi; _close(n) ends the batch at n rows (= the last row_hi).  Completes like the
 * progressive form: pbft_verify_poll_rows reports each chunk's bitmap words as they land (also while the batch is
 * open); pbft_verify_wait refuses an open batch (PBFT_EBUSY).  A failing _piece or _close drops the batch. */
int pbft_verify_votes_open(pbft_ctx *ctx, uint64_t n_cap, uint32_t env_cap, uint64_t *bitmap_out);
int pbft_verify_votes_piece(pbft_ctx *ctx, const uint8_t *rows, uint64_t row_lo, uint64_t row_hi,
                            const uint8_t *envelopes, uint32_t env_lo, uint32_t env_hi);
int pbft_verify_votes_close(pbft_ctx *ctx, uint64_t n);
/* Pinned host memory the context's device (and the node's other GPUs) can DMA from: anonymous pages registered
 * with hipHostRegister (portable; the copy engine reads them faster than later hipHostMalloc buffers).  *out = NULL
 * and PBFT_ENOMEM on failure.  Free with pbft_host_free (it may wait for the device). */
int pbft_host_alloc(pbft_ctx *ctx, size_t bytes, void **out);
int pbft_host_free(pbft_ctx *ctx, void *p);

/* Device-resident form: all pointers are device pointers on the context's
 * device; stream is a hipStream_t (NULL = the context's stream).  Enqueues the
 * kernels only.  d_R / d_S 16-byte aligned; d_msg must stay readable for
 * N*msg_stride + 16 bytes.  A context's workspace is reused by every launch:
 * launches of one context must be ordered (one stream, or events between
 * streams) -- use pbft_verify_ctx_clone for independent concurrent streams.
 * Capturable into a hipGraph after pbft_verify_reserve. */
int pbft_verify_batch_device(pbft_ctx *ctx, const uint8_t *d_R, const uint8_t *d_S, const uint16_t *d_key_idx,
                             const uint8_t *d_msg, uint32_t msg_len, uint32_t msg_stride, uint64_t N,
                             uint64_t *d_bitmap, void *stream);

/* Pipelined device form (a stream of rounds): the one-lane-per-signature kernel of this batch runs on
 * `stream`, its batch-inversion finish (which writes d_bitmap) on `finish_stream` after an event, so the
 * next call's kernel on `stream` overlaps this finish and whatever the caller enqueues after it on
 * finish_stream (e.g. the RCCL all-gather of the bitmaps).  The context alternates two workspace halves: a
 * call waits, on `stream`, for the finish of the call two back.  d_bitmap is complete in finish_stream
 * order.  Small batches (latency mode) run whole on `stream` and finish_stream waits for them.  The
 * streams must differ; pbft_last_kernel_ms reports the `stream` kernel. */
int pbft_verify_batch_device_pipelined(pbft_ctx *ctx, const uint8_t *d_R, const uint8_t *d_S,
                                       const uint16_t *d_key_idx, const uint8_t *d_msg, uint32_t msg_len,
                                       uint32_t msg_stride, uint64_t N, uint64_t *d_bitmap, void *stream,
                                       void *finish_stream);

/* Votes form of a round batch: a PBFT window's Prepares / Commits sign only (kind, view, seq, digest), so the
 * n_env distinct 85-byte envelopes of the batch (one per (kind, seq) of its windows; pbft_envelope) are passed
 * once and signature i names its envelope: envelopes[env_idx[i]].  70 bytes per signature cross PCIe instead
 * of 151.  env_idx[i] >= n_env is bit 0.  Blocking, host buffers (chunked H2D overlapped with the kernels). */
int pbft_verify_votes(pbft_ctx *ctx, const uint8_t *R, const uint8_t *S, const uint16_t *key_idx,
                      const uint32_t *env_idx, const uint8_t *envelopes, uint32_t n_env, uint64_t N,
                      uint64_t *bitmap_out);
/* Device-resident votes form; d_envelopes readable for n_env * 85 + 16 bytes.  Enqueue only.  Both votes forms
 * first expand each envelope's share of the SHA-512 (block 2's message schedule, 512 B per envelope) into a
 * context buffer that grows on first use for a bigger table (so not first called inside a stream capture). */
int pbft_verify_votes_device(pbft_ctx *ctx, const uint8_t *d_R, const uint8_t *d_S, const uint16_t *d_key_idx,
                             const uint32_t *d_env_idx, const uint8_t *d_envelopes, uint32_t n_env, uint64_t N,
                             uint64_t *d_bitmap, void *stream);

/* Pre-size the verify workspace (~230 bytes of HBM per signature) for batches
 * of up to max_n signatures, so that later launches allocate nothing (required
 * before capturing pbft_verify_batch_device into a hipGraph). */
int pbft_verify_reserve(pbft_ctx *ctx, uint64_t max_n);

/* Request digests over N variable-length byte strings packed in `data`:
 * item i is data[offsets[i] .. offsets[i] + lens[i]).  out: N x 64 (Blake2b-512)
 * or N x 32 (SHA-256) bytes.  Blocking, host buffers. */
int pbft_digest_blake2b512(pbft_ctx *ctx, const uint8_t *data, const uint64_t *offsets, const uint32_t *lens,
                           uint64_t N, uint8_t *out);
int pbft_digest_sha256(pbft_ctx *ctx, const uint8_t *data, const uint64_t *offsets, const uint32_t *lens,
                       uint64_t N, uint8_t *out);

/* RFC 8032 batch signing: seeds[n_seeds][32] secret seeds; signature i signs
 * msg[i][0..msg_len) with seeds[seed_idx[i]].  Writes R[N][32], S[N][32];
 * pub (optional) receives the n_seeds public keys.  Blocking, host buffers. */
int pbft_sign_batch(pbft_ctx *ctx, const uint8_t *seeds, uint32_t n_seeds, const uint16_t *seed_idx,
                    const uint8_t *msg, uint32_t msg_len, uint32_t msg_stride, uint64_t N, uint8_t *R,
                    uint8_t *S, uint8_t *pub);

/* Tuning options of one context (defaults are chosen by batch size / free HBM):
 *   PBFT_OPT_SPLIT_BELOW          batches below this many signatures use the 4-lanes-per-signature latency
 *                                 kernel (default 12288; env PBFT_SPLIT_BELOW)
 *   PBFT_OPT_FINISH_WIDTH         signatures per lane of the batch-inversion finish kernel: 1, 2, 4, 8 or 16
 *                                 (0 = by batch size)
 *   PBFT_OPT_KEY_TABLE_BUDGET_MB  HBM budget for the replica key tables at the next pbft_verify_set_keys
 *                                 (0 = env PBFT_KEY_TABLE_BUDGET_MB or 70 % of the free HBM); selects the key
 *                                 comb plan
 *   PBFT_OPT_FINISH_TREE          cross-lane levels of the finish's batch inversion: 0 (one inversion per lane)
 *                                 or 4 (the compiled product tree: one inversion per 16-lane row; 6, the per-wave
 *                                 tree, is a build-time A/B and returns PBFT_EINVAL); any
 *                                 other value = by batch size
 *   PBFT_OPT_LAT_SPLIT            lanes per signature of the latency-mode kernel: 4 or 8; any other value = by
 *                                 batch size (8 up to 8,192 signatures, else 4)
 *   PBFT_OPT_FINISH_WAVES         product-tree finish compiled for 1 wave per SIMD (widths 1-16, X/Y/Z prefetched)
 *                                 or 2 (widths 1, 2, 4, 8; width 1 prefetched); any other value = by batch size
 *   PBFT_OPT_KERNEL_TIMING        1: two HIP events bracket every launch for pbft_last_kernel_ms; 0 (default since
 *                                 r05: the two event records cost ~7.5 us per launch, 4.5 % of an 8-GPU shard): none,
 *                                 and pbft_last_kernel_ms returns -1
 *   PBFT_OPT_COMB_PAIR            1: one-lane batches run the comb with two waves per 64 signatures (a hashing
 *                                 wave and a base-point wave, joined by one extended addition); 0: one wave per
 *                                 64 signatures; any other value = by batch size (pairs up to 98,304 signatures,
 *                                 where one wave per 64 signatures leaves SIMDs short of waves; env
 *                                 PBFT_COMB_PAIR) */
#define PBFT_OPT_SPLIT_BELOW 1
#define PBFT_OPT_FINISH_WIDTH 2
#define PBFT_OPT_KEY_TABLE_BUDGET_MB 3
#define PBFT_OPT_FINISH_TREE 4
#define PBFT_OPT_LAT_SPLIT 5
#define PBFT_OPT_KERNEL_TIMING 7
#define PBFT_OPT_FINISH_WAVES 8
/* (9, 12, 14, 15: options of variants measured slower and removed in r06 -- now PBFT_EINVAL) */
#define PBFT_OPT_COMB_PAIR 10
/* Testing: the next pbft_verify_update_keys on this context fails at a chosen point -- 1: before anything is written
 * (as if its scratch allocation failed: the key set is unchanged), 2: after the updated keys' tables were written
 * (their key_ok is cleared in the shared key set, so every context holding it rejects them); 0: off. */
#define PBFT_OPT_FAULT_INJECT 11
/* 1: the one-lane comb (chain form, 85-byte messages, >= 2^16 signatures) runs 8-wave blocks whose two waves per
 * SIMD trade priorities so that they progress together (instead of oldest-first); 0: 4-wave blocks; any other
 * value (default; env PBFT_COMB_PRIO) = by batch size: 8-wave blocks where they fit one per CU (the 131k shard). */
#define PBFT_OPT_COMB_PRIO 13
int pbft_verify_set_option(pbft_ctx *ctx, int option, uint64_t value);

/* Diagnostics */
const char *pbft_last_error(void);
const char *pbft_build_info(void); /* kernel windows, arch, version */
/* Comb windows in use: wb (base point, build-time) and wa (the installed key
 * set's window, chosen by pbft_verify_set_keys; 0 before it), key count. */
int pbft_verify_ctx_info(pbft_ctx *ctx, uint32_t *wb, uint32_t *wa, uint32_t *n_keys);
/* Device time of the last verify kernel launched by this context, in ms
 * (HIP events on the launch stream). */
float pbft_last_kernel_ms(pbft_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* PBFT_VERIFY_H */
