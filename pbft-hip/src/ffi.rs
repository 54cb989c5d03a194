//! Raw bindings of the C ABI in `include/pbft_verify.h`, `include/pbft_replica.h` and
//! `include/pbft_wire.h` (exported by libpbft_verify.so).  One declaration per C entry
//! point, same names and argument order; no logic here.
//!
//! NOT COMPILED IN THIS REPOSITORY (no Rust toolchain in the image); kept in sync with the
//! headers, whose every symbol `tests/test_abi.py` checks the built library exports.
#![allow(non_camel_case_types)]
use std::os::raw::{c_char, c_int, c_void};

#[repr(C)]
pub struct pbft_ctx {
    _private: [u8; 0],
}
#[repr(C)]
pub struct pbft_replica {
    _private: [u8; 0],
}
#[repr(C)]
pub struct pbft_multi {
    _private: [u8; 0],
}

/// Pinned host staging of one votes-form batch (pbft_verify_votes_stage): filled in place, then submitted.
/// Rows of `row_stride` (PBFT_VOTES_ROW_BYTES = 72) bytes: row i's signature at `sig + i * row_stride`, its key
/// index and envelope index at the same offset from `key_idx` / `env_idx` (as bytes).
#[repr(C)]
pub struct pbft_votes_staging {
    pub sig: *mut u8,
    pub key_idx: *mut u16,
    pub env_idx: *mut u32,
    pub envelopes: *mut u8,
    pub row_stride: u32,
}

pub const PBFT_VOTES_ROW_BYTES: usize = 72;
pub const PBFT_VOTES_ROW_KEY: usize = 64;
pub const PBFT_VOTES_ROW_ENV: usize = 68;

pub const PBFT_OK: c_int = 0;
pub const PBFT_EINVAL: c_int = -1;
pub const PBFT_EHIP: c_int = -2;
pub const PBFT_ENOKEYS: c_int = -3;
pub const PBFT_ENOMEM: c_int = -4;
pub const PBFT_ENODEV: c_int = -5;
pub const PBFT_EBUSY: c_int = -6;

pub const PBFT_OPT_SPLIT_BELOW: c_int = 1;
pub const PBFT_OPT_FINISH_WIDTH: c_int = 2;
pub const PBFT_OPT_KEY_TABLE_BUDGET_MB: c_int = 3;
pub const PBFT_OPT_FINISH_TREE: c_int = 4;
pub const PBFT_OPT_LAT_SPLIT: c_int = 5;
pub const PBFT_OPT_KERNEL_TIMING: c_int = 7;
pub const PBFT_OPT_FINISH_WAVES: c_int = 8;
pub const PBFT_OPT_COMB_PAIR: c_int = 10;
pub const PBFT_OPT_FAULT_INJECT: c_int = 11;
pub const PBFT_OPT_COMB_PRIO: c_int = 13;
pub const PBFT_MAX_REPLICA_CTX: u32 = 16;

pub const PBFT_KIND_PREPREPARE: u8 = 0;
pub const PBFT_KIND_PREPARE: u8 = 1;
pub const PBFT_KIND_COMMIT: u8 = 2;
pub const PBFT_ENVELOPE_BYTES: usize = 85;
pub const PBFT_EVENT_PREPARED: u32 = 1;
pub const PBFT_EVENT_COMMITTED_LOCAL: u32 = 2;
pub const PBFT_EVENT_PRE_PREPARED: u32 = 3;
pub const PBFT_PEER_ID_BYTES: usize = 38;
pub const PBFT_RECORD_BYTES: usize = 160;

#[repr(C)]
#[derive(Clone, Copy, Debug, Default, PartialEq, Eq)]
pub struct pbft_round_event {
    pub view: u64,
    pub seq: u64,
    pub kind: u32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct pbft_replica_stats {
    pub pushed: u64,
    pub verified: u64,
    pub accepted: u64,
    pub rejected_sig: u64,
    pub rejected_digest: u64,
    pub rejected_view: u64,
    pub duplicates: u64,
    pub batches: u64,
    pub rejected_watermark: u64,
    pub rejected_signer: u64,
    pub dropped_flood: u64,
    pub windows_gc: u64,
    pub low_watermark: u64,
    pub live_windows: u64,
    pub submit_ns: u64,
    pub apply_ns: u64,
}

/// Phases of the last push_many / flush (pbft_replica_get_timings; host clock, ns).
#[repr(C)]
#[derive(Debug, Default, Clone, Copy)]
pub struct pbft_replica_timings {
    pub push_checks_ns: u64,
    pub push_windows_ns: u64,
    pub push_rows_ns: u64,
    pub submit_segs_ns: u64,
    pub submit_launch_ns: u64,
    pub wait_ns: u64,
    pub apply_partial_ns: u64,
    pub apply_final_ns: u64,
    pub gc_ns: u64,
    pub polls: u64,
    pub early_pieces: u64,
    pub early_piece_ns: u64,
    pub early_last_rows: u64,
    pub push_checks_end_min_ns: u64,
    pub push_rows_start_max_ns: u64,
    pub push_rows_end_min_ns: u64,
}

/// Phases of the last pbft_verify_set_keys / pbft_verify_update_keys (host wall time, ms).
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct pbft_key_stats {
    pub total_ms: f64,
    pub meminfo_ms: f64,
    pub free_ms: f64,
    pub alloc_ms: f64,
    pub build_ms: f64,
    pub keys_built: u32,
    pub reused: u32,
    pub table_bytes: u64,
}

#[repr(C)]
pub struct pbft_wire_msg {
    pub kind: u32,
    pub view: u64,
    pub seq: u64,
    pub digest: [u8; 64],
    pub digest_ok: u32,
    pub has_sig: u32,
    pub replica: u32,
    pub sig: [u8; 64],
    pub operation: *const c_char,
    pub operation_len: u32,
    pub timestamp: u64,
    pub client: [c_char; 64],
}

pub type pbft_batch_verify_fn = extern "C" fn(
    user: *mut c_void,
    r: *const u8,
    s: *const u8,
    key_idx: *const u16,
    msg: *const u8,
    msg_len: u32,
    msg_stride: u32,
    n: u64,
    bitmap_out: *mut u64,
) -> c_int;
pub type pbft_votes_submit_fn = extern "C" fn(
    user: *mut c_void,
    sig: *const u8,
    key_idx: *const u16,
    env_idx: *const u32,
    envelopes: *const u8,
    n_env: u32,
    n: u64,
    bitmap_out: *mut u64,
) -> c_int;
pub type pbft_votes_poll_fn = extern "C" fn(user: *mut c_void) -> c_int;
pub type pbft_digest_fn =
    extern "C" fn(user: *mut c_void, op: *const u8, op_len: u32, digest_out: *mut u8) -> c_int;

#[link(name = "pbft_verify")]
extern "C" {
    // ---- include/pbft_verify.h
    pub fn pbft_verify_ctx_create(device: c_int, out: *mut *mut pbft_ctx) -> c_int;
    pub fn pbft_verify_ctx_destroy(ctx: *mut pbft_ctx) -> c_int;
    pub fn pbft_verify_set_keys(ctx: *mut pbft_ctx, a: *const u8, n: u32, key_ok: *mut u8) -> c_int;
    pub fn pbft_verify_update_keys(ctx: *mut pbft_ctx, idx: *const u32, a: *const u8, m: u32,
                                   key_ok: *mut u8) -> c_int;
    pub fn pbft_verify_key_stats(ctx: *mut pbft_ctx, out: *mut pbft_key_stats) -> c_int;
    pub fn pbft_verify_revoke_keys(ctx: *mut pbft_ctx, idx: *const u32, m: u32) -> c_int;
    pub fn pbft_verify_key_set_id(ctx: *mut pbft_ctx, id: *mut u64) -> c_int;
    pub fn pbft_verify_ctx_clone(parent: *mut pbft_ctx, out: *mut *mut pbft_ctx) -> c_int;
    pub fn pbft_verify_batch(ctx: *mut pbft_ctx, r: *const u8, s: *const u8, key_idx: *const u16, msg: *const u8,
                             msg_len: u32, msg_stride: u32, n: u64, bitmap_out: *mut u64) -> c_int;
    pub fn pbft_verify_batch_multi(ctxs: *const *mut pbft_ctx, n_ctx: u32, r: *const u8, s: *const u8,
                                   key_idx: *const u16, msg: *const u8, msg_len: u32, msg_stride: u32, n: u64,
                                   bitmap_out: *mut u64) -> c_int;
    pub fn pbft_verify_batch_async(ctx: *mut pbft_ctx, r: *const u8, s: *const u8, key_idx: *const u16,
                                   msg: *const u8, msg_len: u32, msg_stride: u32, n: u64,
                                   bitmap_out: *mut u64) -> c_int;
    pub fn pbft_verify_poll(ctx: *mut pbft_ctx) -> c_int;
    pub fn pbft_verify_wait(ctx: *mut pbft_ctx) -> c_int;
    pub fn pbft_verify_votes_async(ctx: *mut pbft_ctx, r: *const u8, s: *const u8, key_idx: *const u16,
                                   env_idx: *const u32, envelopes: *const u8, n_env: u32, n: u64,
                                   bitmap_out: *mut u64) -> c_int;
    pub fn pbft_verify_votes_stage(ctx: *mut pbft_ctx, n: u64, n_env: u32, out: *mut pbft_votes_staging) -> c_int;
    pub fn pbft_verify_votes_submit(ctx: *mut pbft_ctx, n: u64, n_env: u32, bitmap_out: *mut u64) -> c_int;
    pub fn pbft_verify_votes_submit_begin(ctx: *mut pbft_ctx, n: u64, n_env: u32, bitmap_out: *mut u64) -> c_int;
    pub fn pbft_verify_votes_submit_rows(ctx: *mut pbft_ctx, rows: u64) -> c_int;
    pub fn pbft_verify_poll_rows(ctx: *mut pbft_ctx, rows_done: *mut u64) -> c_int;
    pub fn pbft_verify_votes_submit_host(ctx: *mut pbft_ctx, rows: *const u8, n: u64, envelopes: *const u8,
                                         n_env: u32, bitmap_out: *mut u64) -> c_int;
    pub fn pbft_verify_votes_open(ctx: *mut pbft_ctx, n_cap: u64, env_cap: u32, bitmap_out: *mut u64) -> c_int;
    pub fn pbft_verify_votes_piece(ctx: *mut pbft_ctx, rows: *const u8, row_lo: u64, row_hi: u64,
                                   envelopes: *const u8, env_lo: u32, env_hi: u32) -> c_int;
    pub fn pbft_verify_votes_close(ctx: *mut pbft_ctx, n: u64) -> c_int;
    pub fn pbft_host_alloc(ctx: *mut pbft_ctx, bytes: usize, out: *mut *mut c_void) -> c_int;
    pub fn pbft_host_free(ctx: *mut pbft_ctx, p: *mut c_void) -> c_int;
    pub fn pbft_multi_create(ctxs: *const *mut pbft_ctx, n_ctx: u32, out: *mut *mut pbft_multi) -> c_int;
    pub fn pbft_multi_destroy(m: *mut pbft_multi) -> c_int;
    pub fn pbft_verify_batch_device_multi(m: *mut pbft_multi, d_r: *const *const u8, d_s: *const *const u8,
                                          d_key_idx: *const *const u16, d_msg: *const *const u8, msg_len: u32,
                                          msg_stride: u32, n: *const u64, words_per_rank: u64,
                                          d_bitmap: *const *mut u64) -> c_int;
    pub fn pbft_multi_sync(m: *mut pbft_multi) -> c_int;
    pub fn pbft_verify_batch_device(ctx: *mut pbft_ctx, d_r: *const u8, d_s: *const u8, d_key_idx: *const u16,
                                    d_msg: *const u8, msg_len: u32, msg_stride: u32, n: u64, d_bitmap: *mut u64,
                                    stream: *mut c_void) -> c_int;
    pub fn pbft_verify_batch_device_pipelined(ctx: *mut pbft_ctx, d_r: *const u8, d_s: *const u8,
                                              d_key_idx: *const u16, d_msg: *const u8, msg_len: u32,
                                              msg_stride: u32, n: u64, d_bitmap: *mut u64, stream: *mut c_void,
                                              finish_stream: *mut c_void) -> c_int;
    pub fn pbft_verify_votes(ctx: *mut pbft_ctx, r: *const u8, s: *const u8, key_idx: *const u16,
                             env_idx: *const u32, envelopes: *const u8, n_env: u32, n: u64,
                             bitmap_out: *mut u64) -> c_int;
    pub fn pbft_verify_votes_device(ctx: *mut pbft_ctx, d_r: *const u8, d_s: *const u8, d_key_idx: *const u16,
                                    d_env_idx: *const u32, d_envelopes: *const u8, n_env: u32, n: u64,
                                    d_bitmap: *mut u64, stream: *mut c_void) -> c_int;
    pub fn pbft_verify_reserve(ctx: *mut pbft_ctx, max_n: u64) -> c_int;
    pub fn pbft_digest_blake2b512(ctx: *mut pbft_ctx, data: *const u8, offsets: *const u64, lens: *const u32,
                                  n: u64, out: *mut u8) -> c_int;
    pub fn pbft_digest_sha256(ctx: *mut pbft_ctx, data: *const u8, offsets: *const u64, lens: *const u32, n: u64,
                              out: *mut u8) -> c_int;
    pub fn pbft_sign_batch(ctx: *mut pbft_ctx, seeds: *const u8, n_seeds: u32, seed_idx: *const u16,
                           msg: *const u8, msg_len: u32, msg_stride: u32, n: u64, r: *mut u8, s: *mut u8,
                           pubkeys: *mut u8) -> c_int;
    pub fn pbft_verify_set_option(ctx: *mut pbft_ctx, option: c_int, value: u64) -> c_int;
    pub fn pbft_last_error() -> *const c_char;
    pub fn pbft_build_info() -> *const c_char;
    pub fn pbft_verify_ctx_info(ctx: *mut pbft_ctx, wb: *mut u32, wa: *mut u32, n_keys: *mut u32) -> c_int;
    pub fn pbft_last_kernel_ms(ctx: *mut pbft_ctx) -> f32;

    // ---- include/pbft_replica.h
    pub fn pbft_replica_create(ctx: *mut pbft_ctx, n: u32, self_id: u32, keys: *const u8,
                               out: *mut *mut pbft_replica) -> c_int;
    pub fn pbft_replica_create_multi(ctxs: *const *mut pbft_ctx, n_ctx: u32, n: u32, self_id: u32, keys: *const u8,
                                     out: *mut *mut pbft_replica) -> c_int;
    pub fn pbft_replica_destroy(r: *mut pbft_replica) -> c_int;
    pub fn pbft_replica_update_keys(r: *mut pbft_replica, idx: *const u32, a: *const u8, m: u32,
                                    key_ok: *mut u8) -> c_int;
    pub fn pbft_replica_set_verifier(r: *mut pbft_replica, f: pbft_batch_verify_fn, user: *mut c_void) -> c_int;
    pub fn pbft_replica_set_votes_verifier(r: *mut pbft_replica, submit: pbft_votes_submit_fn,
                                           poll: pbft_votes_poll_fn, user: *mut c_void) -> c_int;
    pub fn pbft_replica_set_digest_fn(r: *mut pbft_replica, f: pbft_digest_fn, user: *mut c_void) -> c_int;
    pub fn pbft_replica_set_log_window(r: *mut pbft_replica, log_window: u64) -> c_int;
    pub fn pbft_envelope(out: *mut u8, kind: u8, view: u64, seq: u64, digest: *const u8);
    pub fn pbft_replica_on_pre_prepare(r: *mut pbft_replica, peer_idx: u32, view: u64, seq: u64, op: *const u8,
                                       op_len: u32, claimed_digest: *const u8, primary_sig: *const u8,
                                       digest_out: *mut u8) -> c_int;
    pub fn pbft_replica_push(r: *mut pbft_replica, kind: u8, view: u64, seq: u64, digest: *const u8, signer: u32,
                             sig: *const u8) -> c_int;
    pub fn pbft_replica_push_frames(r: *mut pbft_replica, peer_idx: u32, stream: *const u8, len: usize,
                                    consumed: *mut u64, pushed: *mut u64, dropped: *mut u64) -> c_int;
    pub fn pbft_replica_push_records(r: *mut pbft_replica, peer_idx: u32, stream: *const u8, len: usize,
                                     consumed: *mut u64, pushed: *mut u64, dropped: *mut u64) -> c_int;
    pub fn pbft_replica_push_many(r: *mut pbft_replica, n: u64, kind: *const u8, view: *const u64, seq: *const u64,
                                  digests: *const u8, signer: *const u32, sigs: *const u8,
                                  queued: *mut u64) -> c_int;
    pub fn pbft_replica_flush_submit(r: *mut pbft_replica, force: c_int, n_rows: *mut u64) -> c_int;
    pub fn pbft_replica_flush_poll(r: *mut pbft_replica, events: *mut pbft_round_event, max_events: u32,
                                   n_events: *mut u32) -> c_int;
    pub fn pbft_replica_in_flight(r: *mut pbft_replica) -> c_int;
    pub fn pbft_replica_flush(r: *mut pbft_replica, force: c_int, events: *mut pbft_round_event, max_events: u32,
                              n_events: *mut u32) -> c_int;
    pub fn pbft_replica_stable_checkpoint(r: *mut pbft_replica, seq: u64) -> c_int;
    pub fn pbft_replica_prepared(r: *mut pbft_replica, view: u64, seq: u64) -> c_int;
    pub fn pbft_replica_committed_local(r: *mut pbft_replica, view: u64, seq: u64) -> c_int;
    pub fn pbft_replica_get_stats(r: *mut pbft_replica, out: *mut pbft_replica_stats) -> c_int;
    pub fn pbft_replica_get_timings(r: *mut pbft_replica, out: *mut pbft_replica_timings) -> c_int;
    pub fn pbft_key_from_peer_id(peer_id: *const u8, len: usize, a: *mut u8) -> c_int;
    pub fn pbft_peer_id_from_key(a: *const u8, peer_id: *mut u8);
    pub fn pbft_key_from_peer_id_b58(text: *const c_char, len: usize, a: *mut u8) -> c_int;
    pub fn pbft_replica_peer_index(r: *mut pbft_replica, peer_id: *const u8, len: usize) -> c_int;

    // ---- include/pbft_wire.h
    pub fn pbft_uvi_encode(v: u64, out: *mut u8) -> usize;
    pub fn pbft_uvi_decode(buf: *const u8, len: usize, value: *mut u64, header_bytes: *mut usize) -> c_int;
    pub fn pbft_wire_encode_json(m: *const pbft_wire_msg, out: *mut c_char, cap: usize, len: *mut usize) -> c_int;
    pub fn pbft_wire_encode_frame(m: *const pbft_wire_msg, out: *mut u8, cap: usize, len: *mut usize) -> c_int;
    pub fn pbft_wire_decode_json(json: *const c_char, len: usize, out: *mut pbft_wire_msg, arena: *mut c_char,
                                 arena_cap: usize) -> c_int;
    pub fn pbft_wire_decode_votes(stream: *const u8, len: usize, n_replicas: u32, max_frames: u64, max_rows: u64,
                                  status: *mut u8, r: *mut u8, s: *mut u8, key_idx: *mut u16, msg: *mut u8,
                                  kind: *mut u8, view: *mut u64, seq: *mut u64, n_frames: *mut u64,
                                  n_rows: *mut u64, consumed: *mut u64) -> c_int;
    pub fn pbft_wire_encode_votes(n: u64, kind: *const u8, view: *const u64, seq: *const u64, digests: *const u8,
                                  replica: *const u32, sigs: *const u8, out: *mut u8, cap: usize,
                                  len: *mut usize) -> c_int;
    pub fn pbft_records_pack(r: *const u8, s: *const u8, key_idx: *const u16, msg: *const u8, msg_stride: u32,
                             n: u64, records: *mut u8) -> c_int;
    pub fn pbft_verify_records_device(ctx: *mut pbft_ctx, d_records: *const u8, n: u64, d_bitmap: *mut u64,
                                      stream: *mut c_void) -> c_int;
    pub fn pbft_verify_records(ctx: *mut pbft_ctx, records: *const u8, n: u64, bitmap_out: *mut u64) -> c_int;
}
