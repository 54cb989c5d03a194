"""In-process n-replica PBFT round driver over the pbft_replica C ABI (test helper).

No network: messages are handed to each replica's state machine directly
(SURVEY.md §4 item 4).  The verifier is either the GPU (ctx) or, for CPU
tests, the C oracle installed through pbft_replica_set_verifier.
"""
import ctypes
import hashlib
import os

import numpy as np

from conftest import ROOT

KIND_PREPREPARE, KIND_PREPARE, KIND_COMMIT = 0, 1, 2
EV_PREPARED, EV_COMMITTED, EV_PRE_PREPARED = 1, 2, 3


class Event(ctypes.Structure):
    _fields_ = [("view", ctypes.c_uint64), ("seq", ctypes.c_uint64), ("kind", ctypes.c_uint32)]


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("pushed", "verified", "accepted", "rejected_sig", "rejected_digest",
                                                "rejected_view", "duplicates", "batches", "rejected_watermark",
                                                "rejected_signer", "dropped_flood", "windows_gc", "low_watermark",
                                                "live_windows", "submit_ns", "apply_ns")]


class Timings(ctypes.Structure):  # include/pbft_replica.h pbft_replica_timings
    _fields_ = [(n, ctypes.c_uint64) for n in ("push_checks_ns", "push_windows_ns", "push_rows_ns", "submit_segs_ns",
                                                "submit_launch_ns", "wait_ns", "apply_partial_ns", "apply_final_ns",
                                                "gc_ns", "polls", "early_pieces", "early_piece_ns", "early_last_rows",
                                                "push_checks_end_min_ns", "push_rows_start_max_ns",
                                                "push_rows_end_min_ns")]


VERIFY_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p)
DIGEST_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p)
# (user, sig[N][64] = R || S, key_idx[N], env_idx[N], envelopes[n_env][85], n_env, N, bitmap_out)
VOTES_SUBMIT_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p)
VOTES_POLL_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)


def lib():
    import pbft_amd
    L = pbft_amd.load()
    vp = ctypes.c_void_p
    L.pbft_replica_create.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p, ctypes.POINTER(vp)]
    L.pbft_replica_create_multi.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p,
                                            ctypes.POINTER(vp)]
    L.pbft_replica_destroy.argtypes = [vp]
    L.pbft_replica_update_keys.argtypes = [vp, vp, ctypes.c_char_p, ctypes.c_uint32, vp]
    L.pbft_replica_set_verifier.argtypes = [vp, VERIFY_FN, vp]
    L.pbft_replica_set_digest_fn.argtypes = [vp, DIGEST_FN, vp]
    L.pbft_replica_on_pre_prepare.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_char_p,
                                              ctypes.c_uint32, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
    L.pbft_replica_push_frames.argtypes = [vp, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t, vp, vp, vp]
    L.pbft_replica_push_records.argtypes = [vp, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t, vp, vp, vp]
    L.pbft_replica_get_timings.argtypes = [vp, ctypes.POINTER(Timings)]
    L.pbft_replica_set_log_window.argtypes = [vp, ctypes.c_uint64]
    L.pbft_replica_stable_checkpoint.argtypes = [vp, ctypes.c_uint64]
    L.pbft_replica_peer_index.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t]
    L.pbft_key_from_peer_id.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    L.pbft_key_from_peer_id_b58.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    L.pbft_peer_id_from_key.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    L.pbft_peer_id_from_key.restype = None
    L.pbft_replica_push.argtypes = [vp, ctypes.c_uint8, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_char_p,
                                    ctypes.c_uint32, ctypes.c_char_p]
    L.pbft_replica_flush.argtypes = [vp, ctypes.c_int, ctypes.POINTER(Event), ctypes.c_uint32,
                                     ctypes.POINTER(ctypes.c_uint32)]
    L.pbft_replica_prepared.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint64]
    L.pbft_replica_committed_local.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint64]
    L.pbft_replica_get_stats.argtypes = [vp, ctypes.POINTER(Stats)]
    L.pbft_replica_set_votes_verifier.argtypes = [vp, VOTES_SUBMIT_FN, VOTES_POLL_FN, vp]
    L.pbft_replica_push_many.argtypes = [vp, ctypes.c_uint64, vp, vp, vp, vp, vp, vp, vp]
    L.pbft_replica_flush_submit.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
    L.pbft_replica_flush_poll.argtypes = [vp, ctypes.POINTER(Event), ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    L.pbft_replica_in_flight.argtypes = [vp]
    L.pbft_envelope.argtypes = [ctypes.c_char_p, ctypes.c_uint8, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_char_p]
    return L


def oracle():
    o = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    vp = ctypes.c_void_p
    o.oracle_verify_batch.argtypes = [vp, ctypes.c_uint32, vp, vp, vp, vp, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint64, vp, ctypes.c_int]
    o.oracle_sign.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
    o.oracle_public_key.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    return o


def seeds(n, tag=1):
    return [hashlib.sha512(b"pbft-key" + tag.to_bytes(8, "little") + i.to_bytes(8, "little")).digest()[:32]
            for i in range(n)]


class AsyncOracleVerifier:
    """Asynchronous votes-form verifier (pbft_replica_set_votes_verifier) backed by the C oracle on a worker thread:
    submit expands envelopes[env_idx[i]] per signature and starts the thread, poll reports it done.  What a
    replica's flush_submit / flush_poll see from the GPU, without a GPU."""

    def __init__(self, cluster, threads=4):
        import threading
        self.c, self.threads, self._t, self._lock = cluster, threads, None, threading.Lock()
        self.submit_cb = VOTES_SUBMIT_FN(self._submit)
        self.poll_cb = VOTES_POLL_FN(self._poll)
        self.batches = 0

    def install(self, rep):
        assert self.c.L.pbft_replica_set_votes_verifier(rep, self.submit_cb, self.poll_cb, None) == 0

    def _submit(self, user, SIG, K, I, E, n_env, N, out):
        import threading
        assert self._t is None
        n = int(N)
        sig = np.ctypeslib.as_array(ctypes.cast(SIG, ctypes.POINTER(ctypes.c_uint8)), (n * 64,)).reshape(n, 64)
        Rn = np.ascontiguousarray(sig[:, :32])
        Sn = np.ascontiguousarray(sig[:, 32:])
        Kn = np.ctypeslib.as_array(ctypes.cast(K, ctypes.POINTER(ctypes.c_uint16)), (n,)).copy()
        In = np.ctypeslib.as_array(ctypes.cast(I, ctypes.POINTER(ctypes.c_uint32)), (n,)).copy()
        En = np.ctypeslib.as_array(ctypes.cast(E, ctypes.POINTER(ctypes.c_uint8)), (int(n_env) * 85,)).copy()
        M = np.zeros((n + 1, 85), np.uint8)
        M[:n] = En.reshape(-1, 85)[In]
        acc = np.zeros(n, np.uint8)
        self.batches += 1

        def work():
            self.c.o.oracle_verify_batch(self.c.keys_np.ctypes.data, self.c.n, Rn.ctypes.data, Sn.ctypes.data,
                                         Kn.ctypes.data, M.ctypes.data, 85, 85, n, acc.ctypes.data, self.threads)
        self._t = (threading.Thread(target=work), acc, out, n)
        self._t[0].start()
        return 0

    def _poll(self, user):
        if self._t is None:
            return 1
        th, acc, out, n = self._t
        if th.is_alive():
            return 0
        th.join()
        bits = np.packbits(np.concatenate([acc, np.zeros((-n) % 64, np.uint8)]), bitorder="little")
        ctypes.memmove(out, bits.ctypes.data, len(bits))
        self._t = None
        return 1


class Cluster:
    """n replicas sharing one key set; signer(seed, msg) -> 64-byte signature."""

    def __init__(self, n, ctx=None, use_oracle_verifier=True, tag=1):
        self.L = lib()
        self.o = oracle()
        self.n = n
        self.seeds = seeds(n, tag)
        pk = []
        for s in self.seeds:
            b = ctypes.create_string_buffer(32)
            self.o.oracle_public_key(b, s)
            pk.append(b.raw)
        self.keys = b"".join(pk)
        self.keys_np = np.frombuffer(self.keys, dtype=np.uint8).copy()
        self._cbs = []
        self.reps = []
        for i in range(n):
            r = ctypes.c_void_p()
            assert self.L.pbft_replica_create(ctx, n, i, self.keys, ctypes.byref(r)) == 0
            if use_oracle_verifier:
                vf = VERIFY_FN(self._oracle_verify)
                df = DIGEST_FN(self._digest)
                self._cbs += [vf, df]
                self.L.pbft_replica_set_verifier(r, vf, None)
                self.L.pbft_replica_set_digest_fn(r, df, None)
            self.reps.append(r)

    def _oracle_verify(self, user, R, S, K, M, msg_len, stride, N, out):
        acc = np.zeros(N, dtype=np.uint8)
        rc = self.o.oracle_verify_batch(self.keys_np.ctypes.data, self.n, R, S, K, M, msg_len, stride, N,
                                        acc.ctypes.data, 4)
        bits = np.packbits(np.concatenate([acc, np.zeros((-N) % 64, np.uint8)]), bitorder="little")
        ctypes.memmove(out, bits.ctypes.data, len(bits))
        return rc

    def _digest(self, user, op, op_len, out):
        data = ctypes.string_at(op, op_len) if op_len else b""
        ctypes.memmove(out, hashlib.blake2b(data, digest_size=64).digest(), 64)
        return 0

    def sign(self, i, kind, view, seq, digest):
        env = ctypes.create_string_buffer(85)
        self.L.pbft_envelope(env, kind, view, seq, digest)
        sig = ctypes.create_string_buffer(64)
        self.o.oracle_sign(sig, self.seeds[i], env.raw, 85)
        return sig.raw

    def flush(self, i, force=0, max_events=4096):
        ev = (Event * max_events)()
        ne = ctypes.c_uint32()
        assert self.L.pbft_replica_flush(self.reps[i], force, ev, max_events, ctypes.byref(ne)) == 0
        return [(e.view, e.seq, e.kind) for e in ev[: ne.value]]

    def flush_submit(self, i, force=0):
        n = ctypes.c_uint64()
        rc = self.L.pbft_replica_flush_submit(self.reps[i], force, ctypes.byref(n))
        assert rc == 0, rc
        return n.value

    def flush_poll(self, i, max_events=4096):
        """None while the batch is in flight, else the delivered events."""
        ev = (Event * max_events)()
        ne = ctypes.c_uint32()
        rc = self.L.pbft_replica_flush_poll(self.reps[i], ev, max_events, ctypes.byref(ne))
        assert rc >= 0, rc
        return None if rc == 0 else [(e.view, e.seq, e.kind) for e in ev[: ne.value]]

    def flush_async(self, i, force=0, max_events=4096):
        """flush_submit, then poll until done (yielding, as an event loop would)."""
        import time
        self.flush_submit(i, force)
        while True:
            evs = self.flush_poll(i, max_events)
            if evs is not None:
                return evs
            time.sleep(0.0005)

    def primary(self, view=1):
        return view % self.n

    def pre_prepare(self, i, view, seq, op, digest=None, sig=None, peer=None):
        """Deliver the primary's signed PrePrepare for (view, seq) to replica i over the connection of replica
        `peer` (default: the view's primary, its legitimate sender)."""
        d = hashlib.blake2b(op, digest_size=64).digest() if digest is None else digest
        if sig is None:
            sig = self.sign(self.primary(view), KIND_PREPREPARE, view, seq, d)
        if peer is None:
            peer = self.primary(view)
        return self.L.pbft_replica_on_pre_prepare(self.reps[i], peer, view, seq, op, len(op), d, sig, None)

    def stats(self, i):
        s = Stats()
        self.L.pbft_replica_get_stats(self.reps[i], ctypes.byref(s))
        return {k: getattr(s, k) for k, _ in Stats._fields_}

    def close(self):
        for r in self.reps:
            self.L.pbft_replica_destroy(r)


class PhaseSim:
    """Phase-ordered PBFT rounds over an in-process network (SURVEY.md §3 S2-S4 in Castro-Liskov order):
    the primary multicasts a signed PrePrepare; a replica sends its Prepare only after the PRE_PREPARED event and
    its Commit only after PREPARED.  `silent` replicas never send anything; `forgers` send, before every honest
    vote, a garbage-signature vote under each honest replica's id (`pbft_replica_push` with a spoofed signer:
    what a transport that trusted the frame's field would deliver).  Flushes are never forced."""

    def __init__(self, cluster, silent=(), forgers=(), op=b"testOperation"):
        self.c, self.silent, self.forgers, self.op = cluster, set(silent), set(forgers), op
        self.D = hashlib.blake2b(op, digest_size=64).digest()
        self.inbox = {i: [] for i in range(cluster.n)}
        self.events = {i: [] for i in range(cluster.n)}

    def honest(self):
        return [i for i in range(self.c.n) if i not in self.silent and i not in self.forgers]

    def _multicast(self, src, kind, view, seq):
        sig = self.c.sign(src, kind, view, seq, self.D)
        for dst in range(self.c.n):
            if self.forgers:
                bad = bytes([sig[0] ^ 0x55]) + sig[1:]
                self.inbox[dst].append((kind, view, seq, self.D, src, bad))
            self.inbox[dst].append((kind, view, seq, self.D, src, sig))

    def start(self, view, seqs):
        p = self.c.primary(view)
        assert p not in self.silent
        for q in seqs:
            for i in range(self.c.n):
                assert self.c.pre_prepare(i, view, q, self.op) == 1

    def run(self, max_rounds=20, async_flush=False):
        """Deliver, flush (never forced), react to events; until quiescent.  Returns rounds used.
        async_flush: every replica's flush is flush_submit + flush_poll (non-blocking form)."""
        L = self.c.L
        for rnd in range(max_rounds):
            progressed = False
            for i in range(self.c.n):
                box, self.inbox[i] = self.inbox[i], []
                for kind, view, seq, d, src, sig in box:
                    L.pbft_replica_push(self.c.reps[i], kind, view, seq, d, src, sig)
                    progressed = True
            for i in range(self.c.n):
                if i in self.silent:
                    continue
                for v, q, k in (self.c.flush_async(i) if async_flush else self.c.flush(i)):
                    progressed = True
                    self.events[i].append((v, q, k))
                    if k == EV_PRE_PREPARED:
                        self._multicast(i, KIND_PREPARE, v, q)
                    elif k == EV_PREPARED:
                        self._multicast(i, KIND_COMMIT, v, q)
            if not progressed:
                return rnd
        return max_rounds

    def committed(self, i, view, seqs):
        return all((view, q, EV_COMMITTED) in self.events[i] for q in seqs)
