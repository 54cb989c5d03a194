"""Round batcher + quorum logic (include/pbft_replica.h) on an in-process n-replica cluster.

BASELINE.json configs[0]: the network.json 4-replica (f = 1) cluster, one
"testOperation" request through pre-prepare / prepare / commit (README.md:42),
CPU verify -- the C oracle is installed as the batch verifier, so the host
state machine is tested without a GPU.  Mirrors src/behavior.rs:100-223 and
src/state.rs:40-75 with the paper's 2f / 2f+1 thresholds, the PrePrepare
signature check (TODO src/behavior.rs:127), votes keyed by the authenticated
peer (src/behavior.rs:346, :380) and the h/H watermarks (TODO :154, :192).
"""
import ctypes
import hashlib

import numpy as np
import pytest

from replica_sim import (EV_COMMITTED, EV_PRE_PREPARED, EV_PREPARED, KIND_COMMIT, KIND_PREPARE, KIND_PREPREPARE,
                         Cluster, PhaseSim)

OP = b"testOperation"
D = hashlib.blake2b(OP, digest_size=64).digest()


def run_round(c, byzantine=(), view=1, seq=1, bad_mode="sig"):
    """Everything delivered up front (PrePrepare + both phases), one non-forced flush per replica."""
    n = c.n
    for i in range(n):
        assert c.pre_prepare(i, view, seq, OP) == 1
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
        assert evs[r] == [(1, 1, EV_PRE_PREPARED), (1, 1, EV_PREPARED), (1, 1, EV_COMMITTED)]
        assert c.L.pbft_replica_committed_local(c.reps[r], 1, 1) == 1
        st = c.stats(r)
        # one batch: the PrePrepare + 4 Prepares + 4 Commits; the decided window is GC'd (h = 1)
        assert st["verified"] == 9 and st["accepted"] == 9 and st["batches"] == 1
        assert st["live_windows"] == 0 and st["low_watermark"] == 1 and st["windows_gc"] == 1
    c.close()


@pytest.mark.parametrize("mode", ["sig", "digest"])
def test_one_byzantine_replica_is_tolerated(mode):
    c = Cluster(4)
    evs = run_round(c, byzantine={3}, bad_mode=mode)
    for r in range(3):
        assert (1, 1, EV_COMMITTED) in evs[r], (r, evs[r])
    st = c.stats(0)
    if mode == "sig":
        assert st["rejected_sig"] == 2 and st["accepted"] == 7
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
    L = c.L
    bad = hashlib.blake2b(b"nope", digest_size=64).digest()
    psig = c.sign(c.primary(), KIND_PREPREPARE, 1, 5, D)
    P = c.primary()
    assert L.pbft_replica_on_pre_prepare(r0, P, 1, 5, OP, len(OP), bad, psig, None) == 0   # digest mismatch
    assert L.pbft_replica_on_pre_prepare(r0, 2, 2, 5, OP, len(OP), D, psig, None) == 0     # wrong view (its primary)
    assert c.stats(0)["rejected_view"] == 1
    assert L.pbft_replica_on_pre_prepare(r0, 2, 1, 5, OP, len(OP), D, psig, None) == 0     # not from the primary
    assert c.stats(0)["rejected_signer"] == 1
    assert L.pbft_replica_on_pre_prepare(r0, P, 1, 5, OP, len(OP), D, psig, None) == 1
    assert L.pbft_replica_on_pre_prepare(r0, P, 1, 5, OP, len(OP), D, psig, None) == 0     # duplicate
    sig = c.sign(2, KIND_PREPARE, 1, 5, D)
    assert L.pbft_replica_push(r0, KIND_PREPARE, 1, 5, D, 2, sig) == 1
    assert L.pbft_replica_push(r0, KIND_PREPARE, 1, 5, D, 2, sig) == 0                  # duplicate
    assert L.pbft_replica_push(r0, KIND_COMMIT, 2, 5, D, 2, sig) == 0                   # commit in other view
    assert L.pbft_replica_push(r0, KIND_PREPARE, 1, 5, D, 9, sig) == 0                  # unknown replica
    # the PrePrepare is always verified at once; one backup's Prepare (< 2f = 2) waits
    assert c.flush(0) == [(1, 5, EV_PRE_PREPARED)] and c.stats(0)["verified"] == 1
    assert c.flush(0) == []
    assert c.flush(0, force=1) == [] and c.stats(0)["verified"] == 2                    # deadline flush
    # a second backup's Prepare completes 2f: the sub-window closes on its own count
    assert L.pbft_replica_push(r0, KIND_PREPARE, 1, 5, D, 3, c.sign(3, KIND_PREPARE, 1, 5, D)) == 1
    assert c.flush(0) == [(1, 5, EV_PREPARED)]
    c.close()


@pytest.mark.parametrize("relay_first", [True, False])
def test_relayed_pre_prepares_cannot_fill_the_primarys_slots(relay_first):
    """a backup relays PBFT_MAX_CANDIDATES (4) junk PrePrepares for a predictable seq through
    pbft_replica_on_pre_prepare (the reference dispatcher's PrePrepare arm with its peer_id, src/behavior.rs:304,
    :310-318); they are dropped at the door (rejected_signer), so the primary's real one -- before or after them --
    is queued, verified and reaches PRE_PREPARED with dropped_flood == 0."""
    c = Cluster(4)
    r0 = c.reps[0]
    backup = 2
    assert backup != c.primary()
    junk = [bytes([k]) * 64 for k in range(1, 5)]
    if not relay_first:
        assert c.pre_prepare(0, 1, 7, OP) == 1
    for j in junk:
        assert c.pre_prepare(0, 1, 7, OP, sig=j, peer=backup) == 0
    # the backup may even relay the primary's VALID PrePrepare: still not its connection's to deliver
    assert c.pre_prepare(0, 1, 7, OP, peer=backup) == 0
    if relay_first:
        assert c.pre_prepare(0, 1, 7, OP) == 1
    assert c.flush(0) == [(1, 7, EV_PRE_PREPARED)]
    st = c.stats(0)
    assert st["dropped_flood"] == 0 and st["rejected_signer"] == 5 and st["rejected_sig"] == 0 and st["verified"] == 1
    c.close()


def test_primary_own_pre_prepare_slots_bounded():
    """The flood bound still holds on the primary's own connection (a faulty primary): 4 candidates, the rest
    dropped_flood."""
    c = Cluster(4)
    for k in range(1, 7):
        c.pre_prepare(0, 1, 9, OP, sig=bytes([k]) * 64)
    st = c.stats(0)
    assert st["dropped_flood"] == 2 and st["rejected_signer"] == 0
    assert c.flush(0) == [] and c.stats(0)["rejected_sig"] == 4
    c.close()


def test_forged_pre_prepare_rejected_then_real_one_accepted():
    c = Cluster(4)
    r0 = c.reps[0]
    forged = bytes(64)
    assert c.pre_prepare(0, 1, 1, OP, sig=forged) == 1                 # queued
    not_primary = c.sign(2, KIND_PREPREPARE, 1, 1, D)                  # validly signed, but not by the primary
    assert c.pre_prepare(0, 1, 1, OP, sig=not_primary) == 1
    assert c.flush(0) == [] and c.stats(0)["rejected_sig"] == 2
    assert c.L.pbft_replica_prepared(r0, 1, 1) == 0
    assert c.pre_prepare(0, 1, 1, OP) == 1                             # the primary's
    assert c.flush(0) == [(1, 1, EV_PRE_PREPARED)]
    c.close()


def test_equivocating_primary_first_accepted_digest_wins():
    """Two validly signed PrePrepares with different digests for one (view, seq): the first accepted fixes the
    window (validate_pre_prepare's conflicting-digest rule, src/behavior.rs:144-151); the other is rejected."""
    c = Cluster(4)
    op2 = b"otherOperation"
    assert c.pre_prepare(0, 1, 1, OP) == 1
    assert c.pre_prepare(0, 1, 1, op2) == 1
    assert c.flush(0) == [(1, 1, EV_PRE_PREPARED)]
    assert c.stats(0)["rejected_digest"] == 1
    assert c.pre_prepare(0, 1, 1, op2) == 0                            # conflicting digest, now known
    c.close()


@pytest.mark.parametrize("n,silent,forgers", [(4, {3}, set()), (4, set(), {2}), (7, {5}, {6}), (4, {0}, set())])
def test_phase_ordered_rounds_without_forced_flush(n, silent, forgers):
    """Castro-Liskov phase order: Prepare only after PRE_PREPARED, Commit only after PREPARED; f replicas silent
    or forging honest replicas' ids before every honest vote.  Every honest replica commits every pipelined
    request with no deadline flush, and the decided windows are garbage-collected."""
    c = Cluster(n)
    sim = PhaseSim(c, silent=silent, forgers=forgers)
    seqs = range(1, 9)
    sim.start(1, seqs)
    rounds = sim.run()
    assert rounds < 20
    for i in sim.honest():
        assert sim.committed(i, 1, seqs), (i, sim.events[i])
        st = c.stats(i)
        assert st["live_windows"] == 0 and st["low_watermark"] == 8, st
        assert c.L.pbft_replica_committed_local(c.reps[i], 1, 5) == 1
        if forgers:
            assert st["rejected_sig"] > 0                              # the forged votes were checked, not trusted
        # batching: 8 windows x 3 phases of signatures in a handful of batches
        assert st["batches"] <= 4, st
    c.close()


def test_watermarks_and_checkpoint():
    c = Cluster(4)
    L, r0 = c.L, c.reps[0]
    assert L.pbft_replica_set_log_window(r0, 8) == 0
    sig = c.sign(2, KIND_PREPARE, 1, 9, D)
    assert L.pbft_replica_push(r0, KIND_PREPARE, 1, 9, D, 2, sig) == 0            # seq 9 > h + 8
    assert c.pre_prepare(0, 1, 9, OP) == 0
    assert c.stats(0)["rejected_watermark"] == 2
    for q in (3, 4, 8):
        assert c.pre_prepare(0, 1, q, OP) == 1
    c.flush(0)
    assert c.stats(0)["live_windows"] == 3
    assert L.pbft_replica_stable_checkpoint(r0, 4) == 0                             # h = 4: windows 3, 4 erased
    st = c.stats(0)
    assert st["live_windows"] == 1 and st["low_watermark"] == 4
    assert L.pbft_replica_push(r0, KIND_PREPARE, 1, 9, D, 2, sig) == 1            # now inside (4, 12]
    assert L.pbft_replica_push(r0, KIND_PREPARE, 1, 4, D, 2, sig) == 0            # below h
    assert L.pbft_replica_set_log_window(r0, 0) == -1
    c.close()


def test_candidate_flood_is_bounded():
    c = Cluster(4)
    L, r0 = c.L, c.reps[0]
    good = c.sign(2, KIND_PREPARE, 1, 1, D)
    for j in range(4):
        assert L.pbft_replica_push(r0, KIND_PREPARE, 1, 1, D, 2, bytes([j + 1]) + good[1:]) == 1
    assert L.pbft_replica_push(r0, KIND_PREPARE, 1, 1, D, 2, good) == 0             # 5th candidate dropped
    assert c.stats(0)["dropped_flood"] == 1
    c.flush(0, force=1)
    assert L.pbft_replica_push(r0, KIND_PREPARE, 1, 1, D, 2, good) == 1             # the real one, once room
    c.close()


def test_pipelined_windows_one_batch():
    """Several (view, seq) windows closing together are verified in one batch (config #2 style)."""
    c = Cluster(4)
    seqs = range(1, 9)
    for q in seqs:
        c.pre_prepare(0, 1, q, OP)
    for q in seqs:
        for s in range(4):
            for kind in (KIND_PREPARE, KIND_COMMIT):
                c.L.pbft_replica_push(c.reps[0], kind, 1, q, D, s, c.sign(s, kind, 1, q, D))
    ev = c.flush(0)
    assert sum(e[2] == EV_COMMITTED for e in ev) == 8
    st = c.stats(0)
    assert st["batches"] == 1 and st["verified"] == 72
    c.close()


def test_events_that_do_not_fit_are_reported_next_flush():
    c = Cluster(4)
    for q in (1, 2, 3):
        c.pre_prepare(0, 1, q, OP)
    first = c.flush(0, max_events=2)
    assert first == [(1, 1, EV_PRE_PREPARED), (1, 2, EV_PRE_PREPARED)]
    assert c.flush(0) == [(1, 3, EV_PRE_PREPARED)]
    c.close()


def test_round_from_wire_frames():
    """Votes arrive as UviBytes/JSON frames on authenticated connections (pbft_replica_push_frames): split reads,
    reference-format unsigned votes and a corrupt frame are dropped, a vote whose "replica" field names another
    peer than the connection's is dropped, the signed PrePrepare is accepted; the round prepares and commits."""
    from pbft_amd import wire
    c = Cluster(4)
    L = c.L
    p = c.primary()
    conns = {s: [] for s in range(4)}  # frames per sending peer
    conns[p].append(wire.encode_frame(wire.WireMsg(kind=wire.PREPREPARE, view=1, seq=1, digest=D, operation=OP,
                                                   client="127.0.0.1:9000", replica=p,
                                                   sig=c.sign(p, KIND_PREPREPARE, 1, 1, D))))
    for kind in (KIND_PREPARE, KIND_COMMIT):
        for s in range(4):
            conns[s].append(wire.encode_frame(wire.WireMsg(kind=kind, view=1, seq=1, digest=D, replica=s,
                                                           sig=c.sign(s, kind, 1, 1, D))))
        conns[0].append(wire.encode_frame(wire.WireMsg(kind=kind, view=1, seq=1, digest=D)))        # unsigned
        # peer 3's connection carrying a vote that claims to be replica 0's (validly signed replay)
        conns[3].append(wire.encode_frame(wire.WireMsg(kind=kind, view=1, seq=1, digest=D, replica=0,
                                                       sig=c.sign(0, kind, 1, 1, D))))
    conns[2].append(wire.uvi_encode(3) + b"{x}")
    for r in range(4):
        tot_p = tot_d = 0
        for s in range(4):
            stream = b"".join(conns[s])
            cut = 37 + 11 * r  # a read boundary inside the first frame, then the rest
            buf, rest = stream[:cut], stream[cut:]
            for chunk in (None, rest):
                if chunk is not None:
                    buf += chunk
                used, pushed, dropped = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
                assert L.pbft_replica_push_frames(c.reps[r], s, buf, len(buf), ctypes.byref(used),
                                                  ctypes.byref(pushed), ctypes.byref(dropped)) == 0
                buf = buf[used.value:]
                tot_p += pushed.value
                tot_d += dropped.value
            assert buf == b""
        assert tot_p == 9 and tot_d == 5, (tot_p, tot_d)
        assert c.stats(r)["rejected_signer"] == 2
        evs = c.flush(r)
        assert (1, 1, EV_PREPARED) in evs and (1, 1, EV_COMMITTED) in evs
    c.close()


def _b58(b: bytes) -> str:
    alpha = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"
    n = int.from_bytes(b, "big")
    out = ""
    while n:
        n, r = divmod(n, 58)
        out = alpha[r] + out
    return "1" * (len(b) - len(b.lstrip(b"\0"))) + out


def test_peer_id_binding():
    """libp2p-core 0.31 Ed25519 PeerId = identity multihash of the protobuf key: 00 24 08 01 12 20 || A
    (src/main.rs:39-40); the authenticated connection's PeerId selects the vote's key index."""
    c = Cluster(4)
    L = c.L
    for i in range(4):
        A = c.keys[32 * i: 32 * i + 32]
        pid = ctypes.create_string_buffer(38)
        L.pbft_peer_id_from_key(A, pid)
        assert pid.raw == bytes([0x00, 0x24, 0x08, 0x01, 0x12, 0x20]) + A
        out = ctypes.create_string_buffer(32)
        assert L.pbft_key_from_peer_id(pid.raw, 38, out) == 0 and out.raw == A
        text = _b58(pid.raw)
        assert text.startswith("12D3KooW")                                     # libp2p's Ed25519 PeerId form
        out2 = ctypes.create_string_buffer(32)
        assert L.pbft_key_from_peer_id_b58(text.encode(), len(text), out2) == 0 and out2.raw == A
        assert L.pbft_replica_peer_index(c.reps[0], pid.raw, 38) == i
    bad = bytes([0x00, 0x25, 0x08, 0x01, 0x12, 0x20]) + bytes(32)
    out = ctypes.create_string_buffer(32)
    assert L.pbft_key_from_peer_id(bad, 38, out) == -1                          # wrong prefix
    assert L.pbft_key_from_peer_id(bad[:37], 37, out) == -1                     # wrong length
    assert L.pbft_key_from_peer_id_b58(b"12D3KooW0OIl", 12, out) == -1          # not base58
    stranger = bytes([0x00, 0x24, 0x08, 0x01, 0x12, 0x20]) + bytes(range(32))
    assert L.pbft_replica_peer_index(c.reps[0], stranger, 38) == -1             # not a replica
    c.close()


def test_replica_update_keys_admits_a_new_identity():
    """pbft_replica_update_keys (the reference's add_peer, src/behavior.rs:45-61): replica 3 gets a new identity;
    its new PeerId resolves to index 3, the old one no longer does, and votes signed with the new key verify
    (the oracle verifier is handed the replica's current key set)."""
    import ctypes
    from replica_sim import seeds as mkseeds
    c = Cluster(4)
    L, r0 = c.L, c.reps[0]
    new_seed = mkseeds(1, tag=99)[0]
    pk = ctypes.create_string_buffer(32)
    c.o.oracle_public_key(pk, new_seed)
    old_pid, new_pid = ctypes.create_string_buffer(38), ctypes.create_string_buffer(38)
    L.pbft_peer_id_from_key(c.keys[96:128], old_pid)
    L.pbft_peer_id_from_key(pk.raw, new_pid)
    assert L.pbft_replica_peer_index(r0, old_pid.raw, 38) == 3
    idx = (ctypes.c_uint32 * 1)(3)
    ok = (ctypes.c_uint8 * 1)()
    assert L.pbft_replica_update_keys(r0, idx, pk.raw, 1, ok) == 0
    assert L.pbft_replica_peer_index(r0, new_pid.raw, 38) == 3 and L.pbft_replica_peer_index(r0, old_pid.raw, 38) < 0
    bad = (ctypes.c_uint32 * 2)(1, 1)
    assert L.pbft_replica_update_keys(r0, bad, pk.raw * 2, 2, None) == -1          # repeated index
    assert L.pbft_replica_update_keys(r0, (ctypes.c_uint32 * 1)(4), pk.raw, 1, None) == -1  # out of range
    # the verifier override judges against the cluster's table: give it the new key too
    keys = bytearray(c.keys)
    keys[96:128] = pk.raw
    c.keys_np = np.frombuffer(bytes(keys), np.uint8).copy()
    c.seeds[3] = new_seed
    assert c.pre_prepare(0, 1, 1, OP) == 1
    for s in (2, 3):
        assert L.pbft_replica_push(r0, KIND_PREPARE, 1, 1, D, s, c.sign(s, KIND_PREPARE, 1, 1, D)) == 1
    evs = c.flush(0)
    assert (1, 1, EV_PREPARED) in evs and c.stats(0)["rejected_sig"] == 0
    c.close()


def test_replica_update_keys_refuses_unreachable_and_keeps_duplicates():
    """a new key that a kept slot already holds is refused (one of the two slots would be unreachable by
    PeerId), as are two equal new keys; swapping two slots' keys in one call is allowed; a replica set created with
    a duplicated key keeps the duplicate's other slot mapped when one of them gets a new identity."""
    import ctypes
    from replica_sim import seeds as mkseeds
    c = Cluster(4)
    L = c.L

    def pid_of(k):
        p = ctypes.create_string_buffer(38)
        L.pbft_peer_id_from_key(k, p)
        return p.raw

    def peer_index(r, k):
        return L.pbft_replica_peer_index(r, pid_of(k), 38)

    r0 = c.reps[0]
    k = [c.keys[32 * i: 32 * i + 32] for i in range(4)]
    one = lambda i: (ctypes.c_uint32 * 1)(i)  # noqa: E731
    assert L.pbft_replica_update_keys(r0, one(3), k[1], 1, None) == -1             # slot 1 keeps that key
    fresh = ctypes.create_string_buffer(32)
    c.o.oracle_public_key(fresh, mkseeds(1, tag=98)[0])
    assert L.pbft_replica_update_keys(r0, (ctypes.c_uint32 * 2)(2, 3), fresh.raw * 2, 2, None) == -1  # equal new keys
    assert L.pbft_replica_update_keys(r0, (ctypes.c_uint32 * 2)(1, 2), k[2] + k[1], 2, None) == 0    # a swap
    assert peer_index(r0, k[1]) == 2 and peer_index(r0, k[2]) == 1
    # duplicates at creation: slots 1 and 3 share a key (first index wins); slot 1 gets a new identity -> the
    # shared key now resolves to slot 3, the new one to slot 1
    dup = bytes(k[0] + k[1] + k[2] + k[1])
    r = ctypes.c_void_p()
    assert L.pbft_replica_create(None, 4, 0, dup, ctypes.byref(r)) == 0
    try:
        assert peer_index(r, k[1]) == 1
        assert L.pbft_replica_update_keys(r, one(1), fresh.raw, 1, None) == 0
        assert peer_index(r, k[1]) == 3 and peer_index(r, fresh.raw) == 1
    finally:
        L.pbft_replica_destroy(r)
    c.close()
