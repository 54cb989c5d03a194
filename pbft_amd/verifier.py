"""BatchVerifier: host-side view of the GPU verifier (BASELINE.json north_star).

Mirrors the trait the reference would bind:

    trait BatchVerifier {
        fn submit(&mut self, b: &SigBatch) -> Ticket;
        fn poll(&mut self, t: Ticket) -> Option<Bitmap>;
        fn verify(&mut self, b: &SigBatch) -> Bitmap;   // blocking
    }

It replaces the per-message validators validate_prepare
(src/behavior.rs:159-175) and validate_commit (src/behavior.rs:184-195), whose
signature checks are TODOs (src/behavior.rs:127, :185).  Invalid signatures are
bit 0 in the returned bitmap, never an exception (the reference panics via
.unwrap() at src/behavior.rs:345, :371; the build drops the message instead).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from ._lib import PbftError, check, load


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a is not None and a.size else 0


@dataclass
class SigBatch:
    """Struct-of-arrays batch of one (view, seq) round window (or several)."""

    R: np.ndarray        # (N, 32) uint8
    S: np.ndarray        # (N, 32) uint8
    key_idx: np.ndarray  # (N,) uint16, index into the installed key set
    msg: np.ndarray      # (N, stride) uint8, first msg_len bytes signed
    msg_len: int

    def __post_init__(self):
        self.R = np.ascontiguousarray(self.R, dtype=np.uint8).reshape(-1, 32)
        self.S = np.ascontiguousarray(self.S, dtype=np.uint8).reshape(-1, 32)
        self.key_idx = np.ascontiguousarray(self.key_idx, dtype=np.uint16).reshape(-1)
        n = len(self.R)
        if len(self.S) != n or len(self.key_idx) != n:
            raise ValueError("R, S and key_idx must have the same length")
        m = np.ascontiguousarray(self.msg, dtype=np.uint8)
        if m.ndim == 1:
            m = m.reshape(n, -1) if n else m.reshape(0, max(self.msg_len, 1))
        if m.shape[0] != n or m.shape[1] < self.msg_len:
            raise ValueError("msg must be (N, stride >= msg_len)")
        self.msg = m

    def __len__(self) -> int:
        return len(self.R)


class KeyStats(ctypes.Structure):
    """pbft_key_stats (include/pbft_verify.h): phases of the last set_keys / update_keys."""
    _fields_ = [("total_ms", ctypes.c_double), ("meminfo_ms", ctypes.c_double), ("free_ms", ctypes.c_double),
                ("alloc_ms", ctypes.c_double), ("build_ms", ctypes.c_double), ("keys_built", ctypes.c_uint32),
                ("reused", ctypes.c_uint32), ("table_bytes", ctypes.c_uint64)]


class VotesStaging(ctypes.Structure):
    """pbft_votes_staging (include/pbft_verify.h)."""
    _fields_ = [("sig", ctypes.c_void_p), ("key_idx", ctypes.c_void_p), ("env_idx", ctypes.c_void_p),
                ("envelopes", ctypes.c_void_p), ("row_stride", ctypes.c_uint32)]


def bitmap_to_bool(bitmap: np.ndarray, n: int) -> np.ndarray:
    """LSB-first u64 words -> bool[n]."""
    bits = np.unpackbits(bitmap.view(np.uint8), bitorder="little")
    return bits[:n].astype(bool)


def verify_multi(verifiers, b: "SigBatch") -> np.ndarray:
    """pbft_verify_batch_multi: shard one batch over several contexts (GPUs and/or clones); bitmap words."""
    lib = load()
    n = len(b)
    out = np.zeros((n + 63) // 64, dtype=np.uint64)
    arr = (ctypes.c_void_p * len(verifiers))(*[v._ctx.value for v in verifiers])
    check(lib.pbft_verify_batch_multi(arr, len(verifiers), _ptr(b.R), _ptr(b.S), _ptr(b.key_idx), _ptr(b.msg),
                                      b.msg_len, b.msg.shape[1], n, _ptr(out)))
    return out


class MultiGpu:
    """pbft_multi_create / pbft_verify_batch_device_multi: one context per device of this process, the round's
    bitmap words all-gathered on RCCL (include/pbft_verify.h)."""

    def __init__(self, verifiers):
        self._lib = load()
        self._m = ctypes.c_void_p()
        # the contexts must outlive the communicator (destroy synchronises their streams): hold the verifiers
        self._verifiers = list(verifiers)
        arr = (ctypes.c_void_p * len(verifiers))(*[v._ctx.value for v in verifiers])
        check(self._lib.pbft_multi_create(arr, len(verifiers), ctypes.byref(self._m)))
        self.n = len(verifiers)

    def verify_device(self, d_R, d_S, d_K, d_M, n, words_per_rank, d_bitmaps, msg_len=85, msg_stride=85):
        """Per-rank lists of device pointers / counts; enqueue only (sync() to wait)."""
        P = ctypes.c_void_p * self.n
        check(self._lib.pbft_verify_batch_device_multi(self._m, P(*d_R), P(*d_S), P(*d_K), P(*d_M), msg_len,
                                                       msg_stride, (ctypes.c_uint64 * self.n)(*n), words_per_rank,
                                                       P(*d_bitmaps)))

    def sync(self):
        check(self._lib.pbft_multi_sync(self._m))

    def close(self):
        if self._m:
            self._lib.pbft_multi_destroy(self._m)
            self._m = ctypes.c_void_p()
        self._verifiers = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GpuBatchVerifier:
    """One HIP context (one GPU).  Not thread-safe: one per host thread."""

    def __init__(self, device: int = 0, _parent: "GpuBatchVerifier | None" = None):
        self._lib = load()
        self._ctx = ctypes.c_void_p()
        if _parent is None:
            check(self._lib.pbft_verify_ctx_create(device, ctypes.byref(self._ctx)))
            self.n_keys = 0
        else:
            check(self._lib.pbft_verify_ctx_clone(_parent._ctx, ctypes.byref(self._ctx)))
            device, self.n_keys = _parent.device, _parent.n_keys
        self.device = device
        self._pending = None

    def clone(self) -> "GpuBatchVerifier":
        """Another context (own HIP stream and workspace) sharing this one's tables and key set."""
        return GpuBatchVerifier(_parent=self)

    # -- key set (libp2p identity keys, src/main.rs:39-40) ------------------
    def set_keys(self, keys: np.ndarray) -> np.ndarray:
        keys = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1, 32)
        ok = np.zeros(len(keys), dtype=np.uint8)
        check(self._lib.pbft_verify_set_keys(self._ctx, _ptr(keys), len(keys), _ptr(ok)))
        self.n_keys = len(keys)
        return ok.astype(bool)

    def update_keys(self, idx, keys: np.ndarray) -> np.ndarray:
        """pbft_verify_update_keys: key idx[i] of the installed set becomes keys[i] (only those tables rebuilt);
        returns key_ok of the new keys."""
        idx = np.ascontiguousarray(idx, dtype=np.uint32).reshape(-1)
        keys = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1, 32)
        if len(idx) != len(keys):
            raise ValueError("idx and keys must have the same length")
        ok = np.zeros(len(keys), dtype=np.uint8)
        check(self._lib.pbft_verify_update_keys(self._ctx, _ptr(idx), _ptr(keys), len(keys), _ptr(ok)))
        return ok.astype(bool)

    def key_stats(self) -> dict:
        """Phases of the last set_keys / update_keys (ms), keys built, whether the allocation was reused."""
        st = KeyStats()
        check(self._lib.pbft_verify_key_stats(self._ctx, ctypes.byref(st)))
        return {k: getattr(st, k) for k, _ in KeyStats._fields_}

    # -- BatchVerifier -------------------------------------------------------
    def verify(self, b: SigBatch) -> np.ndarray:
        """Blocking; returns the ceil(N/64) u64 bitmap words."""
        n = len(b)
        out = np.zeros((n + 63) // 64, dtype=np.uint64)
        check(self._lib.pbft_verify_batch(self._ctx, _ptr(b.R), _ptr(b.S), _ptr(b.key_idx), _ptr(b.msg),
                                          b.msg_len, b.msg.shape[1], n, _ptr(out)))
        return out

    def submit(self, b: SigBatch) -> int:
        n = len(b)
        out = np.zeros((n + 63) // 64, dtype=np.uint64)
        check(self._lib.pbft_verify_batch_async(self._ctx, _ptr(b.R), _ptr(b.S), _ptr(b.key_idx), _ptr(b.msg),
                                                b.msg_len, b.msg.shape[1], n, _ptr(out)))
        self._pending = (b, out)  # keep host buffers alive until poll/wait
        return id(out)

    def poll(self, ticket: int):
        if self._pending is None or id(self._pending[1]) != ticket:
            raise PbftError(-1, "unknown ticket")
        if check(self._lib.pbft_verify_poll(self._ctx)) == 1:
            out = self._pending[1]
            self._pending = None
            return out
        return None

    def wait(self, ticket: int) -> np.ndarray:
        if self._pending is None or id(self._pending[1]) != ticket:
            raise PbftError(-1, "unknown ticket")
        check(self._lib.pbft_verify_wait(self._ctx))
        out = self._pending[1]
        self._pending = None
        return out

    def verify_device(self, d_R: int, d_S: int, d_key_idx: int, d_msg: int, msg_len: int, msg_stride: int,
                      n: int, d_bitmap: int, stream: int = 0) -> None:
        """Enqueue on device-resident buffers (raw device pointers)."""
        check(self._lib.pbft_verify_batch_device(self._ctx, d_R, d_S, d_key_idx, d_msg, msg_len, msg_stride, n,
                                                 d_bitmap, stream or None))

    def verify_device_pipelined(self, d_R: int, d_S: int, d_key_idx: int, d_msg: int, msg_len: int,
                                msg_stride: int, n: int, d_bitmap: int, stream: int, finish_stream: int) -> None:
        """Kernel on `stream`, finish (bitmap) on `finish_stream`: the next call's kernel overlaps this finish."""
        check(self._lib.pbft_verify_batch_device_pipelined(self._ctx, d_R, d_S, d_key_idx, d_msg, msg_len, msg_stride,
                                                           n, d_bitmap, stream, finish_stream))

    def reserve(self, max_n: int) -> None:
        """Pre-size the workspace (required before capturing verify_device into a graph)."""
        check(self._lib.pbft_verify_reserve(self._ctx, max_n))

    def verify_votes(self, R, S, key_idx, env_idx, envelopes) -> np.ndarray:
        """pbft_verify_votes: signature i signs envelopes[env_idx[i]] (85 B each); returns bitmap words."""
        R = np.ascontiguousarray(R, np.uint8).reshape(-1, 32)
        S = np.ascontiguousarray(S, np.uint8).reshape(-1, 32)
        K = np.ascontiguousarray(key_idx, np.uint16).reshape(-1)
        I = np.ascontiguousarray(env_idx, np.uint32).reshape(-1)
        E = np.ascontiguousarray(envelopes, np.uint8).reshape(-1, 85)
        n = len(R)
        if not (len(S) == len(K) == len(I) == n):
            raise ValueError("R, S, key_idx, env_idx must have the same length")
        out = np.zeros((n + 63) // 64, dtype=np.uint64)
        check(self._lib.pbft_verify_votes(self._ctx, _ptr(R), _ptr(S), _ptr(K), _ptr(I), _ptr(E), len(E), n, _ptr(out)))
        return out

    def submit_votes(self, R, S, key_idx, env_idx, envelopes) -> int:
        """pbft_verify_votes_async: non-blocking votes form; complete with poll / wait (the library copies
        pageable buffers into its pinned staging, so the arrays may be reused once this returns)."""
        R = np.ascontiguousarray(R, np.uint8).reshape(-1, 32)
        S = np.ascontiguousarray(S, np.uint8).reshape(-1, 32)
        K = np.ascontiguousarray(key_idx, np.uint16).reshape(-1)
        I = np.ascontiguousarray(env_idx, np.uint32).reshape(-1)
        E = np.ascontiguousarray(envelopes, np.uint8).reshape(-1, 85)
        n = len(R)
        if not (len(S) == len(K) == len(I) == n):
            raise ValueError("R, S, key_idx, env_idx must have the same length")
        out = np.zeros((n + 63) // 64, dtype=np.uint64)
        check(self._lib.pbft_verify_votes_async(self._ctx, _ptr(R), _ptr(S), _ptr(K), _ptr(I), _ptr(E), len(E), n,
                                                _ptr(out)))
        self._pending = ((R, S, K, I, E), out)  # (pinned inputs are DMA'd in place: keep them alive)
        return id(out)

    def stage_votes(self, n: int, n_env: int) -> dict:
        """pbft_verify_votes_stage: numpy views of the context's pinned staging for an (n, n_env) votes batch
        (72-byte rows: sig R || S, key_idx, env_idx as strided views of them; envelopes), to be filled in place and
        launched by submit_staged.
        The views are valid only until the next call on this context that uses the staging (another stage_votes,
        or any host-buffer submit / verify): do not touch them afterwards."""
        st = VotesStaging()
        check(self._lib.pbft_verify_votes_stage(self._ctx, n, n_env, ctypes.byref(st)))

        def view(ptr, dtype, shape):
            count = int(np.prod(shape))
            if count == 0:
                return np.zeros(shape, dtype)
            buf = (ctypes.c_uint8 * (count * np.dtype(dtype).itemsize)).from_address(ptr)
            return np.frombuffer(buf, dtype=dtype).reshape(shape)
        # the rows (PBFT_VOTES_ROW_BYTES each: signature, key_idx at 64, env_idx at 68) as one byte array, the
        # three fields as strided views of it
        rs = int(st.row_stride)
        rows = view(st.sig, np.uint8, (n, rs))
        return {"sig": rows[:, :64], "key_idx": rows[:, 64:66].view(np.uint16).reshape(n),
                "env_idx": rows[:, 68:72].view(np.uint32).reshape(n), "rows": rows,
                "envelopes": view(st.envelopes, np.uint8, (n_env, 85))}

    def submit_staged(self, n: int, n_env: int) -> int:
        out = np.zeros((n + 63) // 64, dtype=np.uint64)
        check(self._lib.pbft_verify_votes_submit(self._ctx, n, n_env, _ptr(out)))
        self._pending = (None, out)
        return id(out)

    def verify_votes_device(self, d_R: int, d_S: int, d_key_idx: int, d_env_idx: int, d_envelopes: int,
                            n_env: int, n: int, d_bitmap: int, stream: int = 0) -> None:
        check(self._lib.pbft_verify_votes_device(self._ctx, d_R, d_S, d_key_idx, d_env_idx, d_envelopes, n_env, n,
                                                 d_bitmap, stream or None))

    def verify_records(self, records: np.ndarray) -> np.ndarray:
        """Blocking verify of (N, 160) binary wire records (include/pbft_wire.h); returns bitmap words."""
        rec = np.ascontiguousarray(records, dtype=np.uint8).reshape(-1, 160)
        n = len(rec)
        out = np.zeros((n + 63) // 64, dtype=np.uint64)
        check(self._lib.pbft_verify_records(self._ctx, _ptr(rec), n, _ptr(out)))
        return out

    OPT_SPLIT_BELOW, OPT_FINISH_WIDTH, OPT_KEY_TABLE_BUDGET_MB, OPT_FINISH_TREE, OPT_LAT_SPLIT = 1, 2, 3, 4, 5
    OPT_KERNEL_TIMING = 7
    OPT_FINISH_WAVES = 8
    OPT_COMB_PAIR = 10
    OPT_FAULT_INJECT = 11
    OPT_COMB_PRIO = 13

    def set_option(self, option: int, value: int) -> None:
        """pbft_verify_set_option: latency-mode threshold, finish width, key-table budget (include/pbft_verify.h)."""
        check(self._lib.pbft_verify_set_option(self._ctx, option, value))

    def positions(self) -> tuple[int, int]:
        """(PB, PA): comb positions (= steps) of the base-point plan and of the installed key set's plan."""
        pb, pa, nk = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        check(self._lib.pbft_verify_ctx_info(self._ctx, ctypes.byref(pb), ctypes.byref(pa), ctypes.byref(nk)))
        return pb.value, pa.value

    def last_kernel_ms(self) -> float:
        return float(self._lib.pbft_last_kernel_ms(self._ctx))

    # -- request digests (src/message.rs:209-212) and signing ---------------
    def _pack(self, items):
        lens = np.array([len(x) for x in items], dtype=np.uint32)
        offs = np.zeros(len(items), dtype=np.uint64)
        if len(items):
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        data = np.frombuffer(b"".join(items) + bytes(16), dtype=np.uint8).copy()
        return data, offs, lens

    def blake2b512(self, items) -> np.ndarray:
        data, offs, lens = self._pack(items)
        out = np.zeros((len(items), 64), dtype=np.uint8)
        check(self._lib.pbft_digest_blake2b512(self._ctx, _ptr(data), _ptr(offs), _ptr(lens), len(items), _ptr(out)))
        return out

    def sha256(self, items) -> np.ndarray:
        data, offs, lens = self._pack(items)
        out = np.zeros((len(items), 32), dtype=np.uint8)
        check(self._lib.pbft_digest_sha256(self._ctx, _ptr(data), _ptr(offs), _ptr(lens), len(items), _ptr(out)))
        return out

    def sign(self, seeds: np.ndarray, seed_idx: np.ndarray, msg: np.ndarray, msg_len: int):
        """RFC 8032 signatures; returns (R, S, public_keys)."""
        seeds = np.ascontiguousarray(seeds, dtype=np.uint8).reshape(-1, 32)
        seed_idx = np.ascontiguousarray(seed_idx, dtype=np.uint16).reshape(-1)
        n = len(seed_idx)
        msg = np.ascontiguousarray(msg, dtype=np.uint8).reshape(n, -1) if n else np.zeros((0, 1), np.uint8)
        R = np.zeros((n, 32), dtype=np.uint8)
        S = np.zeros((n, 32), dtype=np.uint8)
        pub = np.zeros((len(seeds), 32), dtype=np.uint8)
        check(self._lib.pbft_sign_batch(self._ctx, _ptr(seeds), len(seeds), _ptr(seed_idx), _ptr(msg), msg_len,
                                        msg.shape[1], n, _ptr(R), _ptr(S), _ptr(pub)))
        return R, S, pub

    def close(self):
        if self._ctx:
            self._lib.pbft_verify_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
