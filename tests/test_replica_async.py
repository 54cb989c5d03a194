"""Non-blocking replica flush (pbft_replica_flush_submit / _poll, include/pbft_replica.h) and the replica fixes of
the round-2 review, on CPU.

The reference runs one single-threaded poll loop (inject_node_event(&mut self) src/behavior.rs:304, poll :416-426),
so the verifier behind the round batcher must be submit + poll, never a blocking call in the loop (SURVEY.md §3
"Threading").  Here the batch goes out in the votes form (one 85-byte envelope per (kind, view, seq, digest), an
envelope index per signature) to an asynchronous verifier installed with pbft_replica_set_votes_verifier: the C
oracle on a worker thread, or -- for the 2^20-signature round -- a scripted verifier whose completion the test
controls, so that "submit returned while the batch is still running" is observed, not timed.
"""
import ctypes
import hashlib
import time

import numpy as np
import pytest

from replica_sim import (EV_COMMITTED, EV_PRE_PREPARED, EV_PREPARED, KIND_COMMIT, KIND_PREPARE, KIND_PREPREPARE,
                         VOTES_POLL_FN, VOTES_SUBMIT_FN, AsyncOracleVerifier, Cluster, Event, PhaseSim)

OP = b"testOperation"
D = hashlib.blake2b(OP, digest_size=64).digest()


def _as(ptr, ctype, n):
    return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctype)), (n,))


class ScriptedVotes:
    """Votes verifier for a synthetic round: signature i is valid iff S[0] is even AND its envelope
    envelopes[env_idx[i]] is the one R encodes (R[0] = kind, R[1:9] = seq LE, R[9:11] = signer LE) -- so the
    votes-form mapping (envelope table + index per row) is checked on every row.  Completion is released by the
    test."""

    def __init__(self):
        self.release = False
        self.job = None
        self.submit_cb = VOTES_SUBMIT_FN(self._submit)
        self.poll_cb = VOTES_POLL_FN(self._poll)
        self.submitted = 0

    def _submit(self, user, SIG, K, I, E, n_env, N, out):
        n = int(N)
        sig = _as(SIG, ctypes.c_uint8, 64 * n).reshape(n, 64)
        self.job = (sig[:, :32].copy(), sig[:, 32].copy(),
                    _as(K, ctypes.c_uint16, n).copy(), _as(I, ctypes.c_uint32, n).copy(),
                    _as(E, ctypes.c_uint8, 85 * int(n_env)).reshape(-1, 85).copy(), out, n)
        self.submitted += 1
        return 0

    def _poll(self, user):
        if self.job is None:
            return 1
        if not self.release:
            return 0
        R, S0, K, I, E, out, n = self.job
        env = E[I]
        ok = (S0 % 2 == 0)
        ok &= env[:, 4] == R[:, 0]
        ok &= (env[:, 13:21] == R[:, 1:9]).all(axis=1)
        ok &= K == R[:, 9].astype(np.uint16) + (R[:, 10].astype(np.uint16) << 8)
        ok &= (env[:, :4] == np.frombuffer(b"PBFT", np.uint8)).all(axis=1)
        bits = np.packbits(np.concatenate([ok.astype(np.uint8), np.zeros((-n) % 64, np.uint8)]), bitorder="little")
        ctypes.memmove(out, bits.ctypes.data, len(bits))
        self.job = None
        return 1


def _digest(seq):
    return hashlib.blake2b(b"op-" + str(seq).encode(), digest_size=64).digest()


def test_flush_submit_of_a_2p20_round_returns_before_poll_reports_done():
    """Config #4's round through ONE replica: n = 256, 2048 seqs x {Prepare, Commit} = 2^20 votes + 2048
    PrePrepares.  flush_submit builds the votes-form batch (4,096 + 2,048 envelopes) and returns while the verifier
    still runs; flush_poll reports 0 until completion, then applies the bitmap: every window prepares and commits
    except the two seeded to miss their quorum."""
    from replica_sim import lib
    L = lib()
    n, seqs = 256, 2048
    keys = bytes(32 * n)
    rep = ctypes.c_void_p()
    assert L.pbft_replica_create(None, n, 0, keys, ctypes.byref(rep)) == 0
    v = ScriptedVotes()
    assert L.pbft_replica_set_votes_verifier(rep, v.submit_cb, v.poll_cb, None) == 0
    digests = {q: _digest(q) for q in range(1, seqs + 1)}
    from replica_sim import DIGEST_FN
    dfn = DIGEST_FN(lambda u, op, ln, out: ctypes.memmove(out, hashlib.blake2b(ctypes.string_at(op, ln),
                                                                                digest_size=64).digest(), 64) and 0)
    assert L.pbft_replica_set_digest_fn(rep, dfn, None) == 0
    primary = 1 % n
    for q in range(1, seqs + 1):
        sig = bytearray(64)
        sig[0] = KIND_PREPREPARE
        sig[1:9] = q.to_bytes(8, "little")
        sig[9:11] = primary.to_bytes(2, "little")
        op = b"op-" + str(q).encode()
        assert L.pbft_replica_on_pre_prepare(rep, primary, 1, q, op, len(op), digests[q], bytes(sig), None) == 1
    # 2^20 votes, in (seq, kind, signer) order, as columns for pbft_replica_push_many
    N = seqs * 2 * n
    seq = np.repeat(np.arange(1, seqs + 1, dtype=np.uint64), 2 * n)
    kind = np.tile(np.repeat(np.array([KIND_PREPARE, KIND_COMMIT], np.uint8), n), seqs)
    signer = np.tile(np.arange(n, dtype=np.uint32), 2 * seqs)
    view = np.ones(N, np.uint64)
    dig = np.frombuffer(b"".join(digests[q] for q in range(1, seqs + 1)), np.uint8).reshape(seqs, 64)
    digs = np.ascontiguousarray(np.repeat(dig, 2 * n, axis=0))
    sigs = np.zeros((N, 64), np.uint8)
    sigs[:, 0] = kind
    sigs[:, 1:9] = seq.view(np.uint8).reshape(N, 8)
    sigs[:, 9] = signer & 0xFF
    sigs[:, 10] = signer >> 8
    sigs[:, 32] = 2  # even: valid
    # seq 7: 100 backups' Prepares invalid (86 valid < 2f = 170) -> never prepares; seq 9: 90 Commits invalid
    # (166 valid < 2f+1 = 171) -> prepares, never commits; plus scattered single invalid votes that do not matter
    bad = ((seq == 7) & (kind == KIND_PREPARE) & (signer >= 2) & (signer < 102)) | \
          ((seq == 9) & (kind == KIND_COMMIT) & (signer < 90)) | (np.arange(N) % 997 == 5)
    sigs[bad, 32] = 1
    q_ = ctypes.c_uint64()
    t = time.perf_counter()
    assert L.pbft_replica_push_many(rep, N, kind.ctypes.data, view.ctypes.data, seq.ctypes.data, digs.ctypes.data,
                                    signer.ctypes.data, sigs.ctypes.data, ctypes.byref(q_)) == 0
    t_push = time.perf_counter() - t
    assert q_.value == N
    rows = ctypes.c_uint64()
    t = time.perf_counter()
    assert L.pbft_replica_flush_submit(rep, 0, ctypes.byref(rows)) == 0
    t_submit = time.perf_counter() - t
    assert rows.value == N + seqs and v.submitted == 1
    assert L.pbft_replica_in_flight(rep) == 1
    ev = (Event * 8192)()
    ne = ctypes.c_uint32()
    # submitted, not done: poll says 0 and delivers nothing; the loop keeps running (and may keep pushing)
    for _ in range(3):
        assert L.pbft_replica_flush_poll(rep, ev, 8192, ctypes.byref(ne)) == 0 and ne.value == 0
    assert L.pbft_replica_flush_submit(rep, 0, ctypes.byref(rows)) == -6  # PBFT_EBUSY: one batch in flight
    v.release = True
    assert L.pbft_replica_flush_poll(rep, ev, 8192, ctypes.byref(ne)) == 1
    evs = [(e.view, e.seq, e.kind) for e in ev[: ne.value]]
    assert [e[:2] for e in evs] == sorted(e[:2] for e in evs)            # (view, seq) order, as delivered
    pre = {q for _, q, k in evs if k == EV_PRE_PREPARED}
    prep = {q for _, q, k in evs if k == EV_PREPARED}
    com = {q for _, q, k in evs if k == EV_COMMITTED}
    assert pre == set(range(1, seqs + 1))
    assert prep == set(range(1, seqs + 1)) - {7}
    assert com == set(range(1, seqs + 1)) - {7, 9}
    assert L.pbft_replica_in_flight(rep) == 0
    from replica_sim import Stats
    st = Stats()
    L.pbft_replica_get_stats(rep, ctypes.byref(st))
    assert st.verified == N + seqs and st.rejected_sig == int(bad.sum()) and st.batches == 1
    assert st.low_watermark == 6  # committed prefix 1..6; seq 7 blocks it
    L.pbft_replica_destroy(rep)
    print(f"2^20 votes: push_many {t_push * 1e3:.0f} ms, flush_submit {t_submit * 1e3:.0f} ms")


@pytest.mark.parametrize("n,silent,forgers", [(4, {3}, set()), (4, set(), {2}), (7, {5}, {6})])
def test_phase_ordered_rounds_through_async_flush(n, silent, forgers):
    """The Castro-Liskov phase-ordered simulation with every flush non-blocking (submit, then poll from the loop)
    and the C oracle verifying on a worker thread: every honest replica commits every request."""
    c = Cluster(n)
    verifiers = [AsyncOracleVerifier(c) for _ in range(n)]
    for i in range(n):
        verifiers[i].install(c.reps[i])
    sim = PhaseSim(c, silent=silent, forgers=forgers)
    seqs = range(1, 7)
    sim.start(1, seqs)
    assert sim.run(async_flush=True) < 20
    for i in sim.honest():
        assert sim.committed(i, 1, seqs), (i, sim.events[i])
        st = c.stats(i)
        assert st["live_windows"] == 0 and st["low_watermark"] == 6
        if forgers:
            assert st["rejected_sig"] > 0
        assert verifiers[i].batches == st["batches"]
    c.close()


def test_votes_pushed_during_flight_go_into_the_next_batch():
    c = Cluster(4)
    v = AsyncOracleVerifier(c)
    v.install(c.reps[0])
    L, r0 = c.L, c.reps[0]
    assert c.pre_prepare(0, 1, 1, OP) == 1
    for s in range(4):
        assert L.pbft_replica_push(r0, KIND_PREPARE, 1, 1, D, s, c.sign(s, KIND_PREPARE, 1, 1, D)) == 1
    assert c.flush_submit(0) == 5
    # in flight: a duplicate of an in-flight vote is a duplicate; the Commits queue for the next batch
    assert L.pbft_replica_push(r0, KIND_PREPARE, 1, 1, D, 2, c.sign(2, KIND_PREPARE, 1, 1, D)) == 0
    for s in range(4):
        assert L.pbft_replica_push(r0, KIND_COMMIT, 1, 1, D, s, c.sign(s, KIND_COMMIT, 1, 1, D)) == 1
    evs = None
    while evs is None:
        evs = c.flush_poll(0)
    assert evs == [(1, 1, EV_PRE_PREPARED), (1, 1, EV_PREPARED)]
    assert c.flush_async(0) == [(1, 1, EV_COMMITTED)]
    st = c.stats(0)
    assert st["batches"] == 2 and st["verified"] == 9 and st["duplicates"] == 1
    c.close()


def test_relayed_pre_prepares_cannot_crowd_out_the_primary():
    """a backup relaying PBFT_MAX_CANDIDATES forged PrePrepares for a predictable seq must
    not fill the window's candidate slots before the primary's own PrePrepare arrives.  PrePrepare frames are only
    taken from the primary's connection (the reference receives it from the primary, src/behavior.rs:89-95)."""
    from pbft_amd import wire
    c = Cluster(4)
    L, r0 = c.L, c.reps[0]
    p = c.primary()
    relay = 2

    def frames(peer, blobs):
        buf = b"".join(blobs)
        used, pushed, dropped = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        assert L.pbft_replica_push_frames(r0, peer, buf, len(buf), ctypes.byref(used), ctypes.byref(pushed),
                                          ctypes.byref(dropped)) == 0
        return pushed.value, dropped.value

    forged = [wire.encode_frame(wire.WireMsg(kind=wire.PREPREPARE, view=1, seq=5, digest=D, operation=OP,
                                             client="127.0.0.1:9000", replica=p, sig=bytes([j + 1]) * 64))
              for j in range(4)]
    assert frames(relay, forged) == (0, 4)
    assert c.stats(0)["rejected_signer"] == 4 and c.stats(0)["dropped_flood"] == 0
    real = wire.encode_frame(wire.WireMsg(kind=wire.PREPREPARE, view=1, seq=5, digest=D, operation=OP,
                                          client="127.0.0.1:9000", replica=p, sig=c.sign(p, KIND_PREPREPARE, 1, 5, D)))
    assert frames(relay, [real]) == (0, 1)   # validly signed, but relayed: still not taken from a backup
    assert frames(p, [real]) == (1, 0)       # the primary's own connection
    assert c.flush(0) == [(1, 5, EV_PRE_PREPARED)]
    assert c.stats(0)["rejected_sig"] == 0
    c.close()


def test_events_without_a_buffer_do_not_stall_gc():
    """flushing with no event buffer used to leave windows undecided, so h never advanced and
    the log filled up.  Decisions are recorded regardless; the events wait in the queue for the next flush."""
    c = Cluster(4)
    L, r0 = c.L, c.reps[0]
    assert L.pbft_replica_set_log_window(r0, 4) == 0
    for q in range(1, 9):  # twice the log window: only possible if h advances
        assert c.pre_prepare(0, 1, q, OP) == 1
        for kind in (KIND_PREPARE, KIND_COMMIT):
            for s in range(4):
                assert L.pbft_replica_push(r0, kind, 1, q, D, s, c.sign(s, kind, 1, q, D)) == 1
        ne = ctypes.c_uint32(7)
        assert L.pbft_replica_flush(r0, 0, None, 0, ctypes.byref(ne)) == 0 and ne.value == 0
        assert c.stats(0)["low_watermark"] == q
    evs = c.flush(0)
    assert [e for e in evs if e[2] == EV_COMMITTED] == [(1, q, EV_COMMITTED) for q in range(1, 9)]
    assert len(evs) == 24
    c.close()


def test_checkpointed_seqs_are_not_reported_as_committed_here():
    """after a stable checkpoint at 100 and a local commit of 101, seqs 1..100 were reported
    prepared / committed although this replica never decided them."""
    c = Cluster(4)
    L, r0 = c.L, c.reps[0]
    assert L.pbft_replica_stable_checkpoint(r0, 100) == 0
    assert c.pre_prepare(0, 1, 101, OP) == 1
    for kind in (KIND_PREPARE, KIND_COMMIT):
        for s in range(4):
            assert L.pbft_replica_push(r0, kind, 1, 101, D, s, c.sign(s, kind, 1, 101, D)) == 1
    assert (1, 101, EV_COMMITTED) in c.flush(0)
    assert c.stats(0)["low_watermark"] == 101 and c.stats(0)["live_windows"] == 0
    assert L.pbft_replica_committed_local(r0, 1, 101) == 1 and L.pbft_replica_prepared(r0, 1, 101) == 1
    for q in (1, 50, 100):
        assert L.pbft_replica_committed_local(r0, 1, q) == 0 and L.pbft_replica_prepared(r0, 1, q) == 0
    assert L.pbft_replica_committed_local(r0, 2, 101) == 0  # another view
    c.close()


def test_checkpoint_while_a_batch_is_in_flight():
    """A stable checkpoint that erases a window whose rows are in flight: the rows are skipped on completion."""
    c = Cluster(4)
    v = AsyncOracleVerifier(c)
    v.install(c.reps[0])
    L, r0 = c.L, c.reps[0]
    for q in (1, 2):
        assert c.pre_prepare(0, 1, q, OP) == 1
    assert c.flush_submit(0) == 2
    assert L.pbft_replica_stable_checkpoint(r0, 1) == 0
    evs = None
    while evs is None:
        evs = c.flush_poll(0)
    assert evs == [(1, 2, EV_PRE_PREPARED)]
    assert c.stats(0)["live_windows"] == 1
    c.close()


def test_parallel_push_many_equals_serial_pushes():
    """pbft_replica_push_many of >= 2^14 rows runs on the worker pool (each window's rows on one
    thread, in input order).  On a shuffled adversarial mix -- duplicates, conflicting digests, candidate floods,
    wrong views, unknown signers, out-of-window seqs -- it must leave the replica exactly as the same rows pushed
    one at a time: same counters, same queued count, and the same events and counters after a forced flush."""
    from replica_sim import Stats, lib
    L = lib()
    n, seqs = 64, 300
    rng = np.random.default_rng(41)
    rows = []
    for q in range(1, seqs + 1):
        d, d2 = _digest(q), _digest(q + 10_000)
        for kind in (KIND_PREPARE, KIND_COMMIT):
            for s in range(n):
                rows.append((kind, 1, q, d, s, 0))
            for s in rng.choice(n, 8, replace=False):          # duplicates (same signature bytes)
                rows.append((kind, 1, q, d, int(s), 0))
            for s in rng.choice(n, 4, replace=False):          # conflicting digest from the same signer
                rows.append((kind, 1, q, d2, int(s), 1))
            s = int(rng.integers(n))
            for k in range(6):                                  # flood: 6 distinct candidates, 4 kept
                rows.append((kind, 1, q, d, s, 2 + k))
    for k in range(200):
        rows.append((KIND_PREPARE, 2, 5, _digest(5), 3, 0))     # wrong view
        rows.append((KIND_COMMIT, 1, 7, _digest(7), n + k, 0))  # unknown signer
        rows.append((KIND_PREPARE, 1, 10_000 + k, _digest(9), 3, 0))  # out of the log window
    # the first half of the rows in window order (long runs), the second half shuffled (a run per row)
    half = len(rows) // 2
    rows = rows[:half] + [rows[half + i] for i in rng.permutation(len(rows) - half)]
    N = len(rows)
    assert N >= 1 << 15
    kind = np.array([r[0] for r in rows], np.uint8)
    view = np.array([r[1] for r in rows], np.uint64)
    seq = np.array([r[2] for r in rows], np.uint64)
    digs = np.frombuffer(b"".join(r[3] for r in rows), np.uint8).reshape(N, 64).copy()
    signer = np.array([r[4] for r in rows], np.uint32)
    sigs = np.zeros((N, 64), np.uint8)
    sigs[:, 0] = kind
    sigs[:, 1:9] = seq.view(np.uint8).reshape(N, 8)
    sigs[:, 9:11] = (signer & 0xFFFF).astype(np.uint16).view(np.uint8).reshape(N, 2)
    var = np.array([r[5] for r in rows], np.uint8)
    sigs[:, 32] = 2 * var                       # even: valid under ScriptedVotes
    sigs[:, 33] = var
    sigs[rng.random(N) < 0.05, 32] |= 1         # 5 % invalid signatures
    keys = np.zeros((n, 32), np.uint8).tobytes()

    def make():
        rep = ctypes.c_void_p()
        assert L.pbft_replica_create(None, n, 0, keys, ctypes.byref(rep)) == 0
        return rep

    def stats(rep):
        st = Stats()
        L.pbft_replica_get_stats(rep, ctypes.byref(st))
        return {k: getattr(st, k) for k, _ in Stats._fields_ if not k.endswith("_ns")}

    a, b = make(), make()
    qa, qb = ctypes.c_uint64(), ctypes.c_uint64()
    t = time.perf_counter()
    assert L.pbft_replica_push_many(a, N, kind.ctypes.data, view.ctypes.data, seq.ctypes.data, digs.ctypes.data,
                                    signer.ctypes.data, sigs.ctypes.data, ctypes.byref(qa)) == 0
    t_par = time.perf_counter() - t
    total = 0
    for lo in range(0, N, 1000):   # below the parallel threshold: the serial path
        hi = min(N, lo + 1000)
        assert L.pbft_replica_push_many(b, hi - lo, kind[lo:].ctypes.data, view[lo:].ctypes.data, seq[lo:].ctypes.data,
                                        digs[lo:].ctypes.data, signer[lo:].ctypes.data, sigs[lo:].ctypes.data,
                                        ctypes.byref(qb)) == 0
        total += qb.value
    assert qa.value == total and stats(a) == stats(b), (qa.value, total)
    assert stats(a)["dropped_flood"] > 0 and stats(a)["duplicates"] > 0 and stats(a)["rejected_watermark"] == 200
    evs = {}
    for name, rep in (("a", a), ("b", b)):
        v = ScriptedVotes()
        v.release = True
        assert L.pbft_replica_set_votes_verifier(rep, v.submit_cb, v.poll_cb, None) == 0
        from replica_sim import DIGEST_FN
        dfn = DIGEST_FN(lambda u, op, ln, out: ctypes.memmove(out, hashlib.blake2b(ctypes.string_at(op, ln),
                                                                                    digest_size=64).digest(), 64) and 0)
        assert L.pbft_replica_set_digest_fn(rep, dfn, None) == 0
        for q in range(1, seqs + 1):
            sig = bytearray(64)
            sig[0] = KIND_PREPREPARE
            sig[1:9] = q.to_bytes(8, "little")
            sig[9:11] = (1).to_bytes(2, "little")
            op = b"op-" + str(q).encode()
            assert L.pbft_replica_on_pre_prepare(rep, 1, 1, q, op, len(op), _digest(q), bytes(sig), None) == 1
        ev = (Event * 4096)()
        ne = ctypes.c_uint32()
        assert L.pbft_replica_flush(rep, 1, ev, 4096, ctypes.byref(ne)) == 0
        evs[name] = [(e.view, e.seq, e.kind) for e in ev[: ne.value]]
        v.keep = dfn
    # the same events in the same order (not sorted first), and that order is (view, seq)
    assert evs["a"] == evs["b"] and stats(a) == stats(b)
    assert [e[:2] for e in evs["a"]] == sorted(e[:2] for e in evs["a"])
    assert sum(1 for e in evs["a"] if e[2] == EV_COMMITTED) > seqs // 2
    L.pbft_replica_destroy(a)
    L.pbft_replica_destroy(b)
    print(f"push_many {N} rows: {t_par * 1e3:.1f} ms on the pool")
