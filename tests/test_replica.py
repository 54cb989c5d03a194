"""Round batcher + quorum logic (include/pbft_replica.h) on an in-process 4-replica cluster.

BASELINE.json configs[0]: the network.json 4-replica (f = 1) cluster, one
"testOperation" request through pre-prepare / prepare / commit (README.md:42),
CPU verify -- here the C oracle is installed as the batch verifier, so the
host state machine is tested without a GPU.  Mirrors src/behavior.rs:100-223
and src/state.rs:40-75 with the paper's 2f / 2f+1 thresholds.
"""
import hashlib

import pytest

from replica_sim import EV_COMMITTED, EV_PREPARED, KIND_COMMIT, KIND_PREPARE, Cluster

OP = b"testOperation"
D = hashlib.blake2b(OP, digest_size=64).digest()


def run_round(c, byzantine=(), view=1, seq=1, bad_mode="sig"):
    n = c.n
    for i in range(n):
        assert c.L.pbft_replica_on_pre_prepare(c.reps[i], view, seq, OP, len(OP), D, None) == 1
    # prepare phase: every replica multicasts a signed Prepare (own one included)
    for s in range(n):
        sig = c.sign(s, KIND_PREPARE, view, seq, D)
        dig = D
        if s in byzantine:
            if bad_mode == "sig":
                sig = bytes([sig[0] ^ 1]) + sig[1:]
            else:
                dig = hashlib.blake2b(b"other", digest_size=64).digest()
                sig = c.sign(s, KIND_PREPARE, view, seq, dig)
        for r in range(n):
            c.L.pbft_replica_push(c.reps[r], KIND_PREPARE, view, seq, dig, s, sig)
    # commit phase
    for s in range(n):
        sig = c.sign(s, KIND_COMMIT, view, seq, D)
        if s in byzantine:
            sig = bytes(64) if bad_mode == "sig" else c.sign(s, KIND_COMMIT, view, seq,
                                                             hashlib.blake2b(b"x", digest_size=64).digest())
        for r in range(n):
            c.L.pbft_replica_push(c.reps[r], KIND_COMMIT, view, seq, D, s, sig)
    return [c.flush(r) for r in range(n)]


def test_config1_four_replicas_commit():
    c = Cluster(4)
    evs = run_round(c)
    for r in range(4):
        assert (1, 1, EV_PREPARED) in evs[r] and (1, 1, EV_COMMITTED) in evs[r]
        assert c.L.pbft_replica_committed_local(c.reps[r], 1, 1) == 1
        st = c.stats(r)
        assert st["verified"] == 8 and st["accepted"] == 8 and st["batches"] == 1  # one batch per window
    c.close()


@pytest.mark.parametrize("mode", ["sig", "digest"])
def test_one_byzantine_replica_is_tolerated(mode):
    c = Cluster(4)
    evs = run_round(c, byzantine={3}, bad_mode=mode)
    for r in range(3):
        assert (1, 1, EV_COMMITTED) in evs[r], (r, evs[r])
    st = c.stats(0)
    if mode == "sig":
        assert st["rejected_sig"] == 2 and st["accepted"] == 6
    c.close()


def test_two_byzantine_replicas_block_commit():
    c = Cluster(4)
    evs = run_round(c, byzantine={2, 3})
    for r in range(4):
        assert not any(e[2] == EV_COMMITTED for e in evs[r])
        assert c.L.pbft_replica_committed_local(c.reps[r], 1, 1) == 0
    c.close()


def test_validation_rules():
    c = Cluster(4)
    r0 = c.reps[0]
    bad = hashlib.blake2b(b"nope", digest_size=64).digest()
    assert c.L.pbft_replica_on_pre_prepare(r0, 1, 5, OP, len(OP), bad, None) == 0      # digest mismatch
    assert c.L.pbft_replica_on_pre_prepare(r0, 2, 5, OP, len(OP), D, None) == 0        # wrong view
    assert c.L.pbft_replica_on_pre_prepare(r0, 1, 5, OP, len(OP), D, None) == 1
    sig = c.sign(1, KIND_PREPARE, 1, 5, D)
    assert c.L.pbft_replica_push(r0, KIND_PREPARE, 1, 5, D, 1, sig) == 1
    assert c.L.pbft_replica_push(r0, KIND_PREPARE, 1, 5, D, 1, sig) == 0               # duplicate
    assert c.L.pbft_replica_push(r0, KIND_COMMIT, 2, 5, D, 1, sig) == 0                # commit in other view
    assert c.L.pbft_replica_push(r0, KIND_PREPARE, 1, 5, D, 9, sig) == 0               # unknown replica
    assert c.flush(0) == []                                                            # window still open
    ev = c.flush(0, force=1)                                                           # deadline flush
    assert ev == [] and c.stats(0)["verified"] == 1
    c.close()


def test_pipelined_windows_one_batch():
    """Several (view, seq) windows closing together are verified in one batch (config #2 style)."""
    c = Cluster(4)
    seqs = range(1, 9)
    for q in seqs:
        for i in range(4):
            c.L.pbft_replica_on_pre_prepare(c.reps[i], 1, q, OP, len(OP), D, None)
    for q in seqs:
        for s in range(4):
            for kind in (KIND_PREPARE, KIND_COMMIT):
                sig = c.sign(s, kind, 1, q, D)
                c.L.pbft_replica_push(c.reps[0], kind, 1, q, D, s, sig)
    ev = c.flush(0)
    assert sum(e[2] == EV_COMMITTED for e in ev) == 8
    st = c.stats(0)
    assert st["batches"] == 1 and st["verified"] == 64
    c.close()


def test_round_from_wire_frames():
    """Votes arrive as UviBytes/JSON frames (pbft_replica_push_frames): split reads, reference-format unsigned
    votes, a PrePrepare and a corrupt frame are dropped; the round still prepares and commits (f = 1)."""
    import ctypes
    from pbft_amd import wire
    c = Cluster(4)
    L = c.L
    vp = ctypes.c_void_p
    L.pbft_replica_push_frames.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t, vp, vp, vp]
    for i in range(4):
        assert L.pbft_replica_on_pre_prepare(c.reps[i], 1, 1, OP, len(OP), D, None) == 1
    frames = []
    for kind in (KIND_PREPARE, KIND_COMMIT):
        for s in range(4):
            frames.append(wire.encode_frame(wire.WireMsg(kind=kind, view=1, seq=1, digest=D, replica=s,
                                                         sig=c.sign(s, kind, 1, 1, D))))
        frames.append(wire.encode_frame(wire.WireMsg(kind=kind, view=1, seq=1, digest=D)))  # unsigned
    frames.append(wire.encode_frame(wire.WireMsg(kind=wire.PREPREPARE, view=1, seq=1, digest=D, operation=OP,
                                                 client="127.0.0.1:9000")))
    frames.append(wire.uvi_encode(3) + b"{x}")
    stream = b"".join(frames)
    for r in range(4):
        cut = 37 + 11 * r  # a read boundary inside the first frame, then the rest
        tot_p = tot_d = 0
        buf = stream[:cut]
        rest = stream[cut:]
        for chunk in (None, rest):
            if chunk is not None:
                buf += chunk
            used, pushed, dropped = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
            assert L.pbft_replica_push_frames(c.reps[r], buf, len(buf), ctypes.byref(used), ctypes.byref(pushed),
                                              ctypes.byref(dropped)) == 0
            buf = buf[used.value:]
            tot_p += pushed.value
            tot_d += dropped.value
        assert buf == b"" and tot_p == 8 and tot_d == 4
        evs = c.flush(r)
        assert (1, 1, EV_PREPARED) in evs and (1, 1, EV_COMMITTED) in evs
    c.close()
