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
                                                "live_windows")]


VERIFY_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p)
DIGEST_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p)


def lib():
    import pbft_amd
    L = pbft_amd.load()
    vp = ctypes.c_void_p
    L.pbft_replica_create.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p, ctypes.POINTER(vp)]
    L.pbft_replica_destroy.argtypes = [vp]
    L.pbft_replica_set_verifier.argtypes = [vp, VERIFY_FN, vp]
    L.pbft_replica_set_digest_fn.argtypes = [vp, DIGEST_FN, vp]
    L.pbft_replica_on_pre_prepare.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_char_p,
                                              ctypes.c_uint32, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
    L.pbft_replica_push_frames.argtypes = [vp, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t, vp, vp, vp]
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

    def primary(self, view=1):
        return view % self.n

    def pre_prepare(self, i, view, seq, op, digest=None, sig=None):
        """Deliver the primary's signed PrePrepare for (view, seq) to replica i."""
        d = hashlib.blake2b(op, digest_size=64).digest() if digest is None else digest
        if sig is None:
            sig = self.sign(self.primary(view), KIND_PREPREPARE, view, seq, d)
        return self.L.pbft_replica_on_pre_prepare(self.reps[i], view, seq, op, len(op), d, sig, None)

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

    def run(self, max_rounds=20):
        """Deliver, flush (never forced), react to events; until quiescent.  Returns rounds used."""
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
                for v, q, k in self.c.flush(i):
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
