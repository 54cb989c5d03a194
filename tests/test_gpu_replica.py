"""The pbft_replica state machine with the real GPU verifier and GPU request digest."""
import numpy as np
import pytest

from replica_sim import EV_COMMITTED, Cluster, PhaseSim
from test_replica import run_round

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu_cluster():
    from pbft_amd import GpuBatchVerifier
    v = GpuBatchVerifier(0)
    yield v
    v.close()


def test_gpu_cluster_rounds(gpu_cluster):
    v = gpu_cluster
    c = Cluster(4, ctx=v._ctx, use_oracle_verifier=False)
    assert v.set_keys(np.frombuffer(c.keys, dtype=np.uint8)).all()
    evs = run_round(c, seq=1)
    for r in range(4):
        assert (1, 1, EV_COMMITTED) in evs[r]
    evs = run_round(c, byzantine={3}, seq=2)
    for r in range(3):
        assert (1, 2, EV_COMMITTED) in evs[r]
    evs = run_round(c, byzantine={1, 3}, seq=3)
    assert not any(e[2] == EV_COMMITTED for r in range(4) for e in evs[r])
    c.close()


@pytest.mark.parametrize("n,silent,forgers", [(4, {3}, set()), (7, {5}, {6})])
def test_gpu_phase_ordered_rounds(gpu_cluster, n, silent, forgers):
    """Phase-ordered rounds (Commit only after PREPARED), f silent / id-forging replicas, no forced flush: every
    PrePrepare, Prepare and Commit signature is checked by the GPU kernels, digests by the GPU Blake2b."""
    v = gpu_cluster
    c = Cluster(n, ctx=v._ctx, use_oracle_verifier=False, tag=11)
    assert v.set_keys(np.frombuffer(c.keys, dtype=np.uint8)).all()
    sim = PhaseSim(c, silent=silent, forgers=forgers)
    seqs = range(1, 17)
    sim.start(1, seqs)
    assert sim.run() < 20
    for i in sim.honest():
        assert sim.committed(i, 1, seqs), (i, sim.events[i])
        st = c.stats(i)
        assert st["live_windows"] == 0 and st["low_watermark"] == 16
        if forgers:
            assert st["rejected_sig"] > 0
    c.close()


def test_gpu_forged_pre_prepare_rejected_by_the_kernels(gpu_cluster):
    """VERDICT r02 test gap: the forged / non-primary PrePrepares are rejected by the GPU kernels (not the oracle
    callback), the primary's is then accepted; through the non-blocking flush."""
    from test_replica import D, OP
    from replica_sim import EV_PRE_PREPARED, KIND_PREPREPARE
    v = gpu_cluster
    c = Cluster(4, ctx=v._ctx, use_oracle_verifier=False, tag=13)
    assert v.set_keys(np.frombuffer(c.keys, dtype=np.uint8)).all()
    assert c.pre_prepare(0, 1, 1, OP, sig=bytes(64)) == 1
    assert c.pre_prepare(0, 1, 1, OP, sig=c.sign(2, KIND_PREPREPARE, 1, 1, D)) == 1   # signed by a backup
    forged = bytearray(c.sign(c.primary(), KIND_PREPREPARE, 1, 1, D))
    forged[40] ^= 4
    assert c.pre_prepare(0, 1, 1, OP, sig=bytes(forged)) == 1
    assert c.flush_async(0) == [] and c.stats(0)["rejected_sig"] == 3
    assert c.pre_prepare(0, 1, 1, OP) == 1
    assert c.flush_async(0) == [(1, 1, EV_PRE_PREPARED)]
    c.close()


def test_gpu_relayed_pre_prepares_do_not_crowd_out_the_primary(gpu_cluster):
    """VERDICT r03 item 1 on the GPU: a backup relays 4 forged PrePrepares for seq 1 through
    pbft_replica_on_pre_prepare (its authenticated peer index), then the primary's real one arrives; the relays are
    dropped at the door, and the real one is verified by the kernels and reaches PRE_PREPARED with
    dropped_flood == 0 (the GPU Blake2b computes the digest)."""
    from test_replica import D, OP
    from replica_sim import EV_PRE_PREPARED, KIND_PREPREPARE
    v = gpu_cluster
    c = Cluster(4, ctx=v._ctx, use_oracle_verifier=False, tag=23)
    assert v.set_keys(np.frombuffer(c.keys, dtype=np.uint8)).all()
    for k in range(4):
        forged = bytearray(c.sign(c.primary(), KIND_PREPREPARE, 1, 1, D))
        forged[33 + k] ^= 1
        assert c.pre_prepare(0, 1, 1, OP, sig=bytes(forged), peer=3) == 0
    assert c.pre_prepare(0, 1, 1, OP) == 1
    assert c.flush_async(0) == [(1, 1, EV_PRE_PREPARED)]
    st = c.stats(0)
    assert st["dropped_flood"] == 0 and st["rejected_signer"] == 4 and st["rejected_sig"] == 0
    assert st["verified"] == 1 and st["accepted"] == 1
    c.close()


def test_gpu_phase_ordered_rounds_async_flush(gpu_cluster):
    """The phase-ordered simulation with every flush non-blocking (flush_submit + flush_poll) on the GPU."""
    v = gpu_cluster
    c = Cluster(7, ctx=v._ctx, use_oracle_verifier=False, tag=17)
    assert v.set_keys(np.frombuffer(c.keys, dtype=np.uint8)).all()
    sim = PhaseSim(c, silent={5}, forgers={6})
    seqs = range(1, 9)
    sim.start(1, seqs)
    assert sim.run(async_flush=True) < 20
    for i in sim.honest():
        assert sim.committed(i, 1, seqs), (i, sim.events[i])
        assert c.stats(i)["rejected_sig"] > 0
    c.close()


@pytest.mark.parametrize("n_ctx,direct,tasks,piece,shuffle", [(1, "1", None, None, False), (3, "1", None, None, False),
                                                             (1, "0", None, None, False), (3, "0", None, None, False),
                                                             (1, "1", "1", "4096", False), (3, "1", "64", "65536", True),
                                                             (1, "1", None, None, True)])
def test_gpu_replica_2p20_round(gpu_cluster, n_ctx, direct, tasks, piece, shuffle, monkeypatch):
    """Config #4's round through one replica on the GPU: n = 256, 2048 seqs, 2^20 GPU-signed votes + 2048
    PrePrepares pushed, ONE flush_submit, polled to completion; the windows whose quorum was broken by corrupted votes
    neither prepare nor commit, every other one commits.  n_ctx = 3: pbft_replica_create_multi over the context and
    two clones (a slice of the batch per context, each launched and applied on its own -- one GPU
    here, one per GPU on a node): the same events and counters.  direct "1": the replica's row arena (written at push
    time) goes to the GPU as it is (r05); "0" (PBFT_REPLICA_DIRECT=0): the staging fill.  r06:
    push_many's tasks and early pieces at their extremes (one task per thread / 64; pieces of 4,096 rows: ~260 of
    them, the short one first) and the votes in a shuffled order (tasks no longer in seq order: the pieces' partial
    application waits for a seq-ordered prefix) -- the same events, in order, and counters."""
    monkeypatch.setenv("PBFT_REPLICA_DIRECT", direct)
    if tasks:
        monkeypatch.setenv("PBFT_PUSH_TASKS", tasks)
    if piece:
        monkeypatch.setenv("PBFT_MANY_PIECE", piece)
    import ctypes
    import hashlib
    import time
    from replica_sim import EV_PREPARED, Event, KIND_COMMIT, KIND_PREPARE, KIND_PREPREPARE, lib
    v = gpu_cluster
    L = lib()
    n, seqs = 256, 2048
    seeds = np.stack([np.frombuffer(hashlib.sha512(b"pbft-key" + (19).to_bytes(8, "little") +
                                                   i.to_bytes(8, "little")).digest()[:32], np.uint8)
                      for i in range(n)])
    dig = np.stack([np.frombuffer(hashlib.blake2b(b"op-" + str(q).encode(), digest_size=64).digest(), np.uint8)
                    for q in range(1, seqs + 1)])
    envs = np.zeros((seqs, 3, 85), np.uint8)
    for q in range(1, seqs + 1):
        for kind in (KIND_PREPREPARE, KIND_PREPARE, KIND_COMMIT):
            envs[q - 1, kind] = np.frombuffer(b"PBFT" + bytes([kind]) + (1).to_bytes(8, "little") +
                                              q.to_bytes(8, "little") + dig[q - 1].tobytes(), np.uint8)
    # votes in (seq, kind, signer) order + one PrePrepare per seq signed by the primary (replica 1)
    N = seqs * 2 * n
    seq = np.repeat(np.arange(1, seqs + 1, dtype=np.uint64), 2 * n)
    kind = np.tile(np.repeat(np.array([KIND_PREPARE, KIND_COMMIT], np.uint8), n), seqs)
    signer = np.tile(np.arange(n, dtype=np.uint32), 2 * seqs)
    msg = envs[seq.astype(np.int64) - 1, kind.astype(np.int64)]
    R, S, pub = v.sign(seeds, signer.astype(np.uint16), msg, 85)
    pR, pS, _ = v.sign(seeds, np.full(seqs, 1, np.uint16), envs[:, 0], 85)
    assert v.set_keys(pub).all()
    sigs = np.concatenate([R, S], axis=1)
    bad = ((seq == 7) & (kind == KIND_PREPARE) & (signer >= 2) & (signer < 102)) | \
          ((seq == 9) & (kind == KIND_COMMIT) & (signer < 90)) | (np.arange(N) % 997 == 5)
    sigs[bad, 40] ^= 1
    rep = ctypes.c_void_p()
    clones = [v.clone() for _ in range(n_ctx - 1)]        # (after set_keys: clones share the installed key set)
    ctxs = (ctypes.c_void_p * n_ctx)(v._ctx.value, *[c._ctx.value for c in clones])
    assert L.pbft_replica_create_multi(ctxs, n_ctx, n, 0, pub.tobytes(), ctypes.byref(rep)) == 0
    from replica_sim import DIGEST_FN
    dfn = DIGEST_FN(lambda u, op, ln, out: ctypes.memmove(out, hashlib.blake2b(ctypes.string_at(op, ln),
                                                                                digest_size=64).digest(), 64) and 0)
    assert L.pbft_replica_set_digest_fn(rep, dfn, None) == 0
    for q in range(1, seqs + 1):
        op = b"op-" + str(q).encode()
        assert L.pbft_replica_on_pre_prepare(rep, 1, 1, q, op, len(op), dig[q - 1].tobytes(),
                                             (pR[q - 1].tobytes() + pS[q - 1].tobytes()), None) == 1
    view = np.ones(N, np.uint64)
    digs = np.ascontiguousarray(dig[seq.astype(np.int64) - 1])
    if shuffle:  # (every (seq, kind, signer) votes once: any arrival order gives the same outcome)
        perm = np.random.default_rng(6).permutation(N)
        kind, seq, signer = kind[perm].copy(), seq[perm].copy(), signer[perm].copy()
        digs, sigs = np.ascontiguousarray(digs[perm]), np.ascontiguousarray(sigs[perm])
        bad = bad[perm]
    q_ = ctypes.c_uint64()
    assert L.pbft_replica_push_many(rep, N, kind.ctypes.data, view.ctypes.data, seq.ctypes.data, digs.ctypes.data,
                                    signer.ctypes.data, sigs.ctypes.data, ctypes.byref(q_)) == 0 and q_.value == N
    rows = ctypes.c_uint64()
    t0 = time.perf_counter()
    assert L.pbft_replica_flush_submit(rep, 0, ctypes.byref(rows)) == 0
    t1 = time.perf_counter()
    assert rows.value == N + seqs
    ev = (Event * 8192)()
    ne = ctypes.c_uint32()
    polls = 0
    evs = []   # every poll's events (a progressive batch may deliver some before it is done)
    while True:
        rc = L.pbft_replica_flush_poll(rep, ev, 8192, ctypes.byref(ne))
        assert rc >= 0
        evs += [(e.seq, e.kind) for e in ev[: ne.value]]
        if rc == 1:
            break
        polls += 1
    t2 = time.perf_counter()
    assert [q for q, _ in evs] == sorted(q for q, _ in evs)   # (view, seq) order across the chunks
    assert {q for q, k in evs if k == EV_PREPARED} == set(range(1, seqs + 1)) - {7}
    assert {q for q, k in evs if k == EV_COMMITTED} == set(range(1, seqs + 1)) - {7, 9}
    from replica_sim import Stats
    st = Stats()
    L.pbft_replica_get_stats(rep, ctypes.byref(st))
    assert st.rejected_sig == int(bad.sum()) and st.accepted == N + seqs - int(bad.sum())
    assert st.verified == N + seqs and st.batches == 1
    L.pbft_replica_destroy(rep)
    for c in clones:
        c.close()
    print(f"replica 2^20 ({n_ctx} contexts): submit {(t1 - t0) * 1e3:.1f} ms, submit->done {(t2 - t0) * 1e3:.1f} ms, "
          f"{polls} polls")


def _signed_round(v, seeds, n, seq0, seqs, primary=1):
    """(PrePrepare R||S per seq, vote sigs [N][64], kind, seq, signer, digests [N][64], ops) of a round of n replicas
    over seqs seq0 .. seq0 + seqs - 1, votes in (seq, kind, signer) order, signed on the GPU."""
    import hashlib
    from replica_sim import KIND_COMMIT, KIND_PREPARE
    qs = np.arange(seq0, seq0 + seqs, dtype=np.uint64)
    ops = [b"op-" + str(int(q)).encode() for q in qs]
    dig = np.stack([np.frombuffer(hashlib.blake2b(o, digest_size=64).digest(), np.uint8) for o in ops])
    env = lambda k, q, d: np.frombuffer(b"PBFT" + bytes([k]) + (1).to_bytes(8, "little") +  # noqa: E731
                                        int(q).to_bytes(8, "little") + d.tobytes(), np.uint8)
    N = seqs * 2 * n
    seq = np.repeat(qs, 2 * n)
    kind = np.tile(np.repeat(np.array([KIND_PREPARE, KIND_COMMIT], np.uint8), n), seqs)
    signer = np.tile(np.arange(n, dtype=np.uint32), 2 * seqs)
    base = np.stack([np.stack([env(k, q, dig[j]) for k in (0, 1, 2)]) for j, q in enumerate(qs)])
    msg = base[(seq - seq0).astype(np.int64), kind.astype(np.int64)]
    R, S, _ = v.sign(seeds, signer.astype(np.uint16), msg, 85)
    pR, pS, _ = v.sign(seeds, np.full(seqs, primary, np.uint16), base[:, 0], 85)
    digs = np.ascontiguousarray(dig[(seq - seq0).astype(np.int64)])
    return np.concatenate([pR, pS], 1), np.concatenate([R, S], 1), kind, seq, signer, digs, dig, ops, msg


def test_gpu_replica_single_pushes_early_batch(gpu_cluster):
    """r06: rounds delivered the reference's way -- one message per call: each seq's PrePrepare
    (pbft_replica_on_pre_prepare, its digest by the GPU Blake2b on the replica's own clone of the context) and then its
    votes one pbft_replica_push / one 160-byte record (pbft_replica_push_records) at a time.  From the second round on
    the arena is verified in pieces on the GPU while the votes arrive (the single-message early batch); a PrePrepare's
    digest runs while that batch is open.  Every seq commits but the one whose Prepare quorum was forged away, the
    forged votes are the rejected ones, and the events come in seq order."""
    import ctypes
    import hashlib
    from replica_sim import EV_PREPARED, Event, Stats, Timings, lib
    from pbft_amd import wire
    v = gpu_cluster
    L = lib()
    n, seqs = 64, 600                       # 76,800 votes + 600 PrePrepares per round: 2^16-row pieces
    seeds = np.stack([np.frombuffer(hashlib.sha512(b"pbft-key" + (31).to_bytes(8, "little") +
                                                   i.to_bytes(8, "little")).digest()[:32], np.uint8) for i in range(n)])
    _, _, pub = v.sign(seeds, np.arange(n, dtype=np.uint16), np.zeros((n, 85), np.uint8), 85)
    assert v.set_keys(pub).all()
    rep = ctypes.c_void_p()
    assert L.pbft_replica_create(v._ctx, n, 0, pub.tobytes(), ctypes.byref(rep)) == 0
    ev = (Event * 4096)()
    ne = ctypes.c_uint32()
    st0 = Stats()
    try:
        for rnd, how in enumerate(["push", "push", "records"]):
            seq0 = 1 + rnd * seqs
            pps, sigs, kind, seq, signer, digs, dig, ops, msg = _signed_round(v, seeds, n, seq0, seqs)
            bad = ((seq == seq0 + 7) & (kind == 1) & (signer >= 2) & (signer < 50)) | (np.arange(len(seq)) % 991 == 3)
            sigs[bad, 40] ^= 1
            recs = wire.records_pack(sigs[:, :32], sigs[:, 32:], signer.astype(np.uint16), msg) if how == "records" \
                else None
            used, a, b = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
            for j in range(seqs):
                q = seq0 + j
                assert L.pbft_replica_on_pre_prepare(rep, 1, 1, q, ops[j], len(ops[j]), dig[j].tobytes(),
                                                     pps[j].tobytes(), None) == 1
                for i in range(2 * n * j, 2 * n * (j + 1)):
                    if recs is None:
                        assert L.pbft_replica_push(rep, int(kind[i]), 1, int(seq[i]), digs[i].tobytes(),
                                                   int(signer[i]), sigs[i].tobytes()) == 1
                    else:
                        assert L.pbft_replica_push_records(rep, int(signer[i]), recs[i].ctypes.data, 160,
                                                           ctypes.byref(used), ctypes.byref(a), ctypes.byref(b)) == 0
                        assert used.value == 160 and a.value == 1
            rows = ctypes.c_uint64()
            assert L.pbft_replica_flush_submit(rep, 0, ctypes.byref(rows)) == 0 and rows.value == len(seq) + seqs
            evs = []
            while True:
                rc = L.pbft_replica_flush_poll(rep, ev, len(ev), ctypes.byref(ne))
                assert rc >= 0
                evs += [(e.seq, e.kind) for e in ev[: ne.value]]
                if rc == 1:
                    break
            tm = Timings()
            assert L.pbft_replica_get_timings(rep, ctypes.byref(tm)) == 0
            if rnd:
                assert tm.early_pieces >= 1 and tm.early_last_rows < (1 << 16) + 64, (rnd, tm.early_pieces)
            else:
                assert tm.early_pieces == 0  # (the first round sizes the arena)
            allq = set(range(seq0, seq0 + seqs))
            assert [x for x, _ in evs] == sorted(x for x, _ in evs)
            assert {x for x, k in evs if k == EV_PREPARED} == allq - {seq0 + 7}
            assert {x for x, k in evs if k == EV_COMMITTED} == allq - {seq0 + 7}
            st = Stats()
            L.pbft_replica_get_stats(rep, ctypes.byref(st))
            assert st.rejected_sig - st0.rejected_sig == int(bad.sum())
            assert st.accepted - st0.accepted == len(seq) + seqs - int(bad.sum())
            st0 = st
    finally:
        L.pbft_replica_destroy(rep)


def test_gpu_replica_update_keys_all_or_nothing(gpu_cluster):
    """VERDICT r05 item 4 / ADVICE r05: a replica over two independently created contexts (two key sets, as two GPUs
    of a node); pbft_replica_update_keys fails on the second (PBFT_OPT_FAULT_INJECT 2: after its tables were written).
    Afterwards EVERY context rejects the slot's signatures under the old and the new key (revoked everywhere), the
    PeerId map keeps the old identity, and the other slots verify; a retry installs the new key on both contexts and
    maps its PeerId; a flush over both contexts then accepts the slot's new-key votes in both slices."""
    import ctypes
    import hashlib
    from pbft_amd import GpuBatchVerifier, SigBatch, bitmap_to_bool
    from replica_sim import Event, Stats, lib
    L = lib()
    n, slot = 16, 5
    seeds = np.stack([np.frombuffer(hashlib.sha512(b"pbft-key" + (41).to_bytes(8, "little") +
                                                   i.to_bytes(8, "little")).digest()[:32], np.uint8) for i in range(n)])
    v0 = gpu_cluster
    v1 = GpuBatchVerifier(0)
    rep = ctypes.c_void_p()
    try:
        _, _, pub = v0.sign(seeds, np.arange(n, dtype=np.uint16), np.zeros((n, 85), np.uint8), 85)
        assert v0.set_keys(pub).all() and v1.set_keys(pub).all()
        ctxs = (ctypes.c_void_p * 2)(v0._ctx.value, v1._ctx.value)
        assert L.pbft_replica_create_multi(ctxs, 2, n, 0, pub.tobytes(), ctypes.byref(rep)) == 0
        seeds_new = seeds.copy()
        seeds_new[slot] = np.frombuffer(hashlib.sha512(b"new-key").digest()[:32], np.uint8)
        msg = np.tile(np.frombuffer(b"PBFT\x01" + bytes(80), np.uint8), (4 * n, 1))
        K = np.tile(np.arange(n, dtype=np.uint16), 4)
        Ro, So, _ = v0.sign(seeds, K, msg, 85)
        Rn, Sn, pub_new = v0.sign(seeds_new, K, msg, 85)
        hit = K == slot

        def bits(v, R, S):
            return bitmap_to_bool(v.verify(SigBatch(R, S, K, msg, 85)), len(K))
        v1.set_option(v1.OPT_FAULT_INJECT, 2)
        ok = np.zeros(1, np.uint8)
        idx = np.array([slot], np.uint32)
        assert L.pbft_replica_update_keys(rep, idx.ctypes.data, pub_new[slot].tobytes(), 1, ok.ctypes.data) < 0
        assert ok[0] == 0
        for v in (v0, v1):  # revoked on both: neither key verifies for the slot, every other slot does
            for R, S in ((Ro, So), (Rn, Sn)):
                b = bits(v, R, S)
                assert not b[hit].any() and b[~hit].all()
        pid = ctypes.create_string_buffer(38)
        L.pbft_peer_id_from_key(pub[slot].tobytes(), pid)
        assert L.pbft_replica_peer_index(rep, pid.raw, 38) == slot          # the old identity kept
        L.pbft_peer_id_from_key(pub_new[slot].tobytes(), pid)
        assert L.pbft_replica_peer_index(rep, pid.raw, 38) < 0
        assert L.pbft_replica_update_keys(rep, idx.ctypes.data, pub_new[slot].tobytes(), 1, ok.ctypes.data) == 0
        assert ok[0] == 1
        assert L.pbft_replica_peer_index(rep, pid.raw, 38) == slot
        for v in (v0, v1):
            assert bits(v, Rn, Sn).all()
            b = bits(v, Ro, So)
            assert not b[hit].any() and b[~hit].all()
        # a round over both contexts: 2 x 2^16 votes, the slot voting with its new key in both slices
        pub2 = pub.copy()
        pub2[slot] = pub_new[slot]
        seqs = 2100
        pps, sigs, kind, seq, signer, digs, dig, ops, _ = _signed_round(v0, seeds_new, n, 1, seqs)
        for j in range(seqs):
            assert L.pbft_replica_on_pre_prepare(rep, 1, 1, 1 + j, ops[j], len(ops[j]), dig[j].tobytes(),
                                                 pps[j].tobytes(), None) == 1
        view = np.ones(len(seq), np.uint64)
        qd = ctypes.c_uint64()
        assert L.pbft_replica_push_many(rep, len(seq), kind.ctypes.data, view.ctypes.data, seq.ctypes.data,
                                        digs.ctypes.data, signer.ctypes.data, sigs.ctypes.data, ctypes.byref(qd)) == 0
        ev = (Event * 8192)()
        ne = ctypes.c_uint32()
        assert L.pbft_replica_flush(rep, 0, ev, 8192, ctypes.byref(ne)) == 0
        assert sum(1 for e in ev[: ne.value] if e.kind == EV_COMMITTED) == seqs
        st = Stats()
        L.pbft_replica_get_stats(rep, ctypes.byref(st))
        assert st.rejected_sig == 0 and st.accepted == len(seq) + seqs
    finally:
        if rep:
            L.pbft_replica_destroy(rep)
        v1.close()
