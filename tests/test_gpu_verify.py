"""GPU parity: the HIP kernels vs the oracle, bit-exact (run with -m gpu on an MI355X).

Checked through the C ABI (pbft_amd binds libpbft_verify.so with ctypes):
  * committed golden vectors (18 adversarial classes, 11 message lengths);
  * seeded config-#3 round (n = 64 keys, 2^16 signatures, 1 % adversarial) vs
    the C oracle (oracle/ed25519_oracle.c), and the full-size config-#4 round
    (2^20) through size-independent properties + a popcount/checksum vs the oracle;
  * RFC 8032 signing vs the oracle signer; Blake2b-512 / SHA-256 vs hashlib;
  * API edges: N = 0, 1, 63, 65, out-of-range key index, async submit/poll,
    device-resident entry point with odd strides.
"""
import ctypes
import hashlib
import json
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, golden_batches

pytestmark = pytest.mark.gpu
L = 2**252 + 27742317777372353535851937790883648493
KAT = json.load(open(os.path.join(GOLDEN, "kat.json")))


@pytest.fixture(scope="module")
def gv():
    from pbft_amd import GpuBatchVerifier
    v = GpuBatchVerifier(0)
    yield v
    v.close()


@pytest.fixture(scope="module")
def coracle():
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    vp = ctypes.c_void_p
    lib.oracle_verify_batch.argtypes = [vp, ctypes.c_uint32, vp, vp, vp, vp, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_uint64, vp, ctypes.c_int]
    lib.oracle_sign_batch.argtypes = [vp, vp, vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, vp, vp,
                                      ctypes.c_int]
    lib.oracle_public_key.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    return lib


def oracle_bits(coracle, keys, R, S, key_idx, msg, msg_len):
    n = len(R)
    out = np.zeros(n, dtype=np.uint8)
    msg = np.ascontiguousarray(msg)
    rc = coracle.oracle_verify_batch(keys.ctypes.data, len(keys), R.ctypes.data, S.ctypes.data, key_idx.ctypes.data,
                                     msg.ctypes.data, msg_len, msg.shape[1], n, out.ctypes.data,
                                     min(16, os.cpu_count() or 1))  # the GPU box's CPU share
    assert rc == 0
    return out.astype(bool)


def seeds_for(n, tag=0):
    return np.stack([np.frombuffer(hashlib.sha512(b"pbft-key" + tag.to_bytes(8, "little") +
                                                  i.to_bytes(8, "little")).digest()[:32], dtype=np.uint8)
                     for i in range(n)])


def round_batch(gv, n_keys, n_seq, seq0=1, tag=0):
    """A synthetic PBFT round: every replica signs Prepare + Commit per seq (GPU signer)."""
    seeds = seeds_for(n_keys, tag)
    msgs = []
    for s in range(seq0, seq0 + n_seq):
        d = hashlib.blake2b(b"op-" + str(s).encode(), digest_size=64).digest()
        for kind in (1, 2):
            env = b"PBFT" + bytes([kind]) + (1).to_bytes(8, "little") + s.to_bytes(8, "little") + d
            msgs.extend([env] * n_keys)
    msg = np.frombuffer(b"".join(msgs), dtype=np.uint8).reshape(-1, 85).copy()
    key_idx = np.tile(np.arange(n_keys, dtype=np.uint16), 2 * n_seq)
    R, S, pub = gv.sign(seeds, key_idx, msg, 85)
    return seeds, pub, R, S, key_idx, msg


def adversarial(rng, pub, R, S, key_idx, msg, frac=0.01):
    """Mutate a seeded `frac` of lanes across the §8(d) adversarial classes."""
    R, S, key_idx, msg = R.copy(), S.copy(), key_idx.copy(), msg.copy()
    n = len(R)
    idx = rng.choice(n, size=max(12, int(n * frac)), replace=False)
    so = [bytes.fromhex(h) for h in KAT["small_order_encodings"]]
    nc = [bytes.fromhex(h) for h in KAT["noncanonical_decodable_encodings"]]
    # an encoding that does not decode (y^2 - 1)/(d y^2 + 1) non-square: y = 2 is one
    noc = (2).to_bytes(32, "little")
    for j, i in enumerate(idx):
        c = j % 12
        if c == 0:
            msg[i, rng.integers(85)] ^= 1 << rng.integers(8)
        elif c == 1:
            R[i, rng.integers(32)] ^= 1 << rng.integers(8)
        elif c == 2:
            S[i, rng.integers(32)] ^= 1 << rng.integers(8)  # byte 31 too: bits 253..255
        elif c == 3:
            s = int.from_bytes(S[i].tobytes(), "little") + L
            S[i] = np.frombuffer(s.to_bytes(32, "little"), dtype=np.uint8)
        elif c == 4:
            S[i, 31] |= 0x80
        elif c == 5:
            R[i] = np.frombuffer(noc, dtype=np.uint8)
        elif c == 6:
            R[i] = np.frombuffer(nc[j % len(nc)], dtype=np.uint8)
        elif c == 7:
            R[i] = np.frombuffer(so[j % len(so)], dtype=np.uint8)
        elif c == 8:
            key_idx[i] = (key_idx[i] + 1) % len(pub)
        elif c == 9:
            R[i] = 0
            S[i] = 0
        elif c == 10:
            key_idx[i] = len(pub) + 3  # out of the installed key set
        else:  # s >= 2^253: rejected, and must not gather past the end of the base-point table
            top = (0xff, 0x20, 0x40, 0xe0)[j % 4]
            if top == 0xff:
                S[i] = 0xff
            else:
                S[i, 31] |= top
    return R, S, key_idx, msg, idx


def verify(gv, R, S, key_idx, msg, msg_len):
    from pbft_amd import SigBatch, bitmap_to_bool
    bm = gv.verify(SigBatch(R, S, key_idx, msg, msg_len))
    return bitmap_to_bool(bm, len(R)), bm


def test_golden_bitmaps_bit_exact(gv, golden):
    for ml, b in golden_batches(golden):
        ok = gv.set_keys(b["keys"])
        assert (ok == b["key_ok"].astype(bool)).all(), ml
        got, bm = verify(gv, b["R"], b["S"], b["key_idx"], b["msg"], ml)
        exp = b["expected"].astype(bool)
        bad = np.nonzero(got != exp)[0]
        assert len(bad) == 0, (ml, bad[:10], b["cls"][bad[:10]])
        n = len(b["R"])
        if n % 64:
            assert int(bm[-1]) >> (n % 64) == 0  # bits past N are zero


def test_sign_matches_oracle(gv, coracle):
    rng = np.random.default_rng(1)
    for ml in (0, 1, 47, 85, 111, 200):
        n = 300
        seeds = rng.integers(0, 256, size=(17, 32), dtype=np.uint8)
        idx = rng.integers(0, 17, size=n).astype(np.uint16)
        stride = max(ml, 1)
        msg = rng.integers(0, 256, size=(n, stride), dtype=np.uint8)
        R, S, pub = gv.sign(seeds, idx, msg, ml)
        oR = np.zeros_like(R)
        oS = np.zeros_like(S)
        buf = np.zeros(n * stride + 16, dtype=np.uint8)
        buf[: n * stride] = msg.ravel()
        assert coracle.oracle_sign_batch(seeds.ctypes.data, idx.ctypes.data, buf.ctypes.data, ml, stride, n,
                                         oR.ctypes.data, oS.ctypes.data, 8) == 0
        assert (R == oR).all() and (S == oS).all(), ml
        for j in range(17):
            pk = ctypes.create_string_buffer(32)
            coracle.oracle_public_key(pk, seeds[j].tobytes())
            assert pk.raw == pub[j].tobytes()


def test_config3_round_with_adversarial(gv, coracle):
    """n = 64 replicas (f = 21), 2^16 signatures, 1 % adversarial (BASELINE configs[2])."""
    seeds, pub, R, S, key_idx, msg = round_batch(gv, 64, 512, tag=3)
    assert gv.set_keys(pub).all()
    rng = np.random.default_rng(3)
    R2, S2, K2, M2, idx = adversarial(rng, pub, R, S, key_idx, msg)
    got, _ = verify(gv, R2, S2, K2, M2, 85)
    exp = oracle_bits(coracle, pub, R2, S2, K2, M2, 85)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
    assert not got[idx].any() and got.sum() == len(R) - len(idx)


def test_comb_pair_matches_oracle(gv, coracle):
    """PBFT_OPT_COMB_PAIR (r04): the comb with two waves per 64 signatures (a hashing wave and a base-point wave
    joined by one extended addition) gives the oracle's bits, forced on and off and by batch size, above its
    automatic range (140,800 and the 131k shard), inside it with ragged tails, and for a non-envelope message
    length."""
    seeds, pub, R, S, key_idx, msg = round_batch(gv, 64, 1100, tag=5)        # 140,800 signatures
    assert gv.set_keys(pub).all()
    rng = np.random.default_rng(5)
    R2, S2, K2, M2, idx = adversarial(rng, pub, R, S, key_idx, msg)
    exp = oracle_bits(coracle, pub, R2, S2, K2, M2, 85)
    assert not exp[idx].any()
    try:
        for n in (len(R2), 131072, 65536 + 63, 20000 + 1):
            for mode in (1, 0, 2):
                gv.set_option(gv.OPT_COMB_PAIR, mode)
                got, bm = verify(gv, R2[:n], S2[:n], K2[:n], M2[:n], 85)
                assert (got == exp[:n]).all(), (n, mode, np.nonzero(got != exp[:n])[0][:10])
                if n % 64:
                    assert int(bm[-1]) >> (n % 64) == 0
        # a message length other than the 85-byte envelope (the generic SHA-512 path of the hashing wave)
        n, ml = 40000, 111
        m = rng.integers(0, 256, size=(n, ml), dtype=np.uint8)
        ki = rng.integers(0, 64, size=n).astype(np.uint16)
        Rm, Sm, _ = gv.sign(seeds, ki, m, ml)
        Sm[::501, 5] ^= 4
        e2 = oracle_bits(coracle, pub, Rm, Sm, ki, m, ml)
        for mode in (1, 0):
            gv.set_option(gv.OPT_COMB_PAIR, mode)
            got, _ = verify(gv, Rm, Sm, ki, m, ml)
            assert (got == e2).all() and not got[::501].any(), mode
    finally:
        gv.set_option(gv.OPT_COMB_PAIR, 2)


P = 2**255 - 19


def test_wave_inversion_extremes_on_gpu(gv):
    """The finish's row-wise inversion itself (inv25519.h fe_invert_wave<true>: table divsteps with the scaled zeta,
    unshifted low bits, 24-bit products, the next batch's first read before the carries and the exit test on the
    limbs before the carries), one value per 16-lane row through the library's test hook pbft_debug_invert, equals
    z^(p-2) on the values that stress the divstep count and the limb ranges (powers of two, p - 2^k, all-ones
    patterns, values just below and above p, 0) and on random values of every bit length."""
    from pbft_amd._lib import load
    lib = load()
    lib.pbft_debug_invert.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
    vals = [2**k for k in range(255)] + [P - 2**k for k in range(1, 255)] + [(2**k - 1) for k in range(1, 256)]
    vals += [P - k for k in range(1, 40)] + [P + k for k in range(0, 19)] + [2**255 - 1 - k for k in range(20)]
    vals += [0, 1, 2, 19, 38, (P + 1) // 2, P - 1]
    rnd = random.Random(20261018)
    vals += [rnd.getrandbits(rnd.randrange(1, 256)) for _ in range(20000)]
    vals = [v % 2**255 for v in vals]
    words = np.array([[(v >> (32 * t)) & 0xFFFFFFFF for t in range(8)] for v in vals], dtype=np.uint32)
    out = np.zeros_like(words)
    assert lib.pbft_debug_invert(words.ctypes.data, out.ctypes.data, len(vals)) == 0
    got = [sum(int(w) << (32 * t) for t, w in enumerate(row)) for row in out]
    bad = [(v, g) for v, g in zip(vals, got) if g != pow(v, P - 2, P)]
    assert not bad, f"{len(bad)} of {len(vals)} inverses differ, first: {bad[0]}"



def test_comb_prio_match_oracle(gv, coracle):
    """r05 comb form PBFT_OPT_COMB_PRIO (8-wave blocks whose SIMD-sharing waves trade priorities), forced on and off
    and by size, against the oracle's bits -- at the 131k shard, ragged sizes whose last block is partial, and a size
    with several generations of blocks; the pair comb forced off so that the chain form runs below its threshold
    too.  r06: the rejected variants' options (zero-copy votes 9, spread 12, fused finish 14, staggered hash 15) are
    gone and refused."""
    from pbft_amd import PbftError
    seeds, pub, R, S, key_idx, msg = round_batch(gv, 64, 2100, tag=7)         # 268,800 signatures
    assert gv.set_keys(pub).all()
    rng = np.random.default_rng(7)
    R2, S2, K2, M2, idx = adversarial(rng, pub, R, S, key_idx, msg)
    exp = oracle_bits(coracle, pub, R2, S2, K2, M2, 85)
    assert not exp[idx].any()
    for removed in (9, 12, 14, 15):
        with pytest.raises(PbftError):
            gv.set_option(removed, 1)
    try:
        gv.set_option(gv.OPT_COMB_PAIR, 0)
        for n in (131072, 65536 + 63, 131072 - 256 - 5, 200_003, len(R2)):
            for prio in (2, 1, 0):
                gv.set_option(gv.OPT_COMB_PRIO, prio)
                got, bm = verify(gv, R2[:n], S2[:n], K2[:n], M2[:n], 85)
                assert (got == exp[:n]).all(), (n, prio, np.nonzero(got != exp[:n])[0][:10])
                if n % 64:
                    assert int(bm[-1]) >> (n % 64) == 0
    finally:
        gv.set_option(gv.OPT_COMB_PAIR, 2)
        gv.set_option(gv.OPT_COMB_PRIO, 2)


def test_config4_full_size_properties(gv, coracle):
    """2^20 signatures (BASELINE configs[3] round): size-independent properties + oracle checksum."""
    seeds, pub, R, S, key_idx, msg = round_batch(gv, 256, 2048, tag=4)
    assert gv.set_keys(pub).all()
    got, bm = verify(gv, R, S, key_idx, msg, 85)
    assert got.all()                                    # every honest signature accepted
    rng = np.random.default_rng(4)
    R2, S2, K2, M2, idx = adversarial(rng, pub, R, S, key_idx, msg, frac=0.001)
    got2, bm2 = verify(gv, R2, S2, K2, M2, 85)
    assert set(np.nonzero(~got2)[0].tolist()) == set(idx.tolist())   # exactly the mutated lanes
    got3, bm3 = verify(gv, R2, S2, K2, M2, 85)
    assert (bm3 == bm2).all()                           # idempotent
    # the oracle agrees on a 2^14 slice containing mutated lanes
    sl = slice(int(idx.min()) // 64 * 64, int(idx.min()) // 64 * 64 + 16384)
    exp = oracle_bits(coracle, pub, R2[sl], S2[sl], K2[sl], M2[sl], 85)
    assert (got2[sl] == exp).all()
    # sub-batch sizes that select the other finish configurations (4 and 2 signatures per lane at one wave per
    # SIMD; the full round uses 8 with the tree at two waves per SIMD) and a ragged tail: the same bits as the
    # full-round launch
    for n in (300_007, 65_536 + 63, 4096):
        got4, _ = verify(gv, R2[:n], S2[:n], K2[:n], M2[:n], 85)
        assert (got4 == got2[:n]).all(), n


def test_config4_every_lane_vs_oracle(gv, coracle):
    """the headline round (n = 256 keys, 2048 seqs x {Prepare, Commit} = 2^20 GPU-signed
    envelopes) with every adversarial class at 0.5 %, a small-order key (slot 254) and a mixed-order key (slot 255,
    with Python-built equation-valid and cofactored-only signatures) in the key set: EVERY lane of the SoA path,
    the votes form (host columns and staged rows) and config #5's serving path (16 x 4096-signature batches
    submitted concurrently over 4 cloned contexts, from one thread and from 4 threads) equals the C oracle
    (oracle_verify_batch over all 2^20 lanes).  Slots certified: /root/reference/src/behavior.rs:159-195."""
    import concurrent.futures as cf

    import torch
    import fullround as F
    from pbft_amd import SigBatch, bitmap_to_bool
    seeds, pub, R, S, key_idx, msg = round_batch(gv, 256, 2048, tag=4)
    n = len(R)
    assert n == 1 << 20
    pub2, a = F.install_special_keys(seeds, pub, small_slot=254, mixed_slot=255)
    ok = gv.set_keys(pub2)
    assert ok[:254].all() and not ok[254] and ok[255]
    R1, S1, v_lanes, c_lanes = F.plant_mixed(R, S, key_idx, msg, 85, pub2, a, 255, n_valid=192, n_cofactored=96,
                                             seed=4)
    rng = np.random.default_rng(44)
    R2, S2, K2, M2, idx = adversarial(rng, pub2, R1, S1, key_idx, msg, frac=0.005)
    exp = oracle_bits(coracle, pub2, R2, S2, K2, M2, 85)
    # the construction did what it says (checked on the oracle's bits)
    untouched = np.ones(n, bool)
    untouched[idx] = False
    assert exp[np.setdiff1d(v_lanes, idx)].all() and not exp[c_lanes].any()
    assert not exp[K2 == 254].any() and not exp[idx].any()
    assert exp[untouched & (K2 < 254)].all()
    assert 0.97 * n < exp.sum() < n

    def check(got, what, sl=slice(None)):
        bad = np.nonzero(got != exp[sl])[0]
        assert len(bad) == 0, (what, len(bad), bad[:10])

    got, bm = verify(gv, R2, S2, K2, M2, 85)
    check(got, "soa")
    # votes form: a table of the round's distinct envelopes (mutated messages are envelopes of their own)
    env, inv = np.unique(M2, axis=0, return_inverse=True)
    ei = inv.reshape(-1).astype(np.uint32)
    check(bitmap_to_bool(gv.verify_votes(R2, S2, K2, ei, env), n), "votes")
    st = gv.stage_votes(n, len(env))
    st["sig"][:, :32], st["sig"][:, 32:], st["key_idx"][:], st["env_idx"][:] = R2, S2, K2, ei
    st["envelopes"][:] = env
    check(bitmap_to_bool(gv.wait(gv.submit_staged(n, len(env))), n), "votes staged")
    # config #5: 16 batches of 4096 over 4 clones, four in flight at once
    offs = [int(o) // 64 * 64 for o in np.linspace(0, n - 4096, 16)]
    clones = [gv.clone() for _ in range(4)]
    try:
        pin = lambda x: torch.from_numpy(np.ascontiguousarray(x)).pin_memory().numpy()  # noqa: E731
        PR, PS, PK, PM = pin(R2), pin(S2), pin(K2), pin(M2)
        for g in range(0, 16, 4):
            tickets = []
            for ci, o in enumerate(offs[g:g + 4]):
                sl = slice(o, o + 4096)
                tickets.append((ci, o, clones[ci].submit(SigBatch(PR[sl], PS[sl], PK[sl], PM[sl], 85))))
            while tickets:
                rest = []
                for ci, o, t in tickets:
                    out = clones[ci].poll(t)
                    if out is None:
                        rest.append((ci, o, t))
                    else:
                        check(bitmap_to_bool(out, 4096), ("stream", o), slice(o, o + 4096))
                tickets = rest

        def worker(ci):
            res = []
            for o in offs[ci::4]:
                sl = slice(o, o + 4096)
                res.append((o, bitmap_to_bool(clones[ci].verify(SigBatch(R2[sl], S2[sl], K2[sl], M2[sl], 85)), 4096)))
            return res
        with cf.ThreadPoolExecutor(4) as ex:
            for fut in [ex.submit(worker, ci) for ci in range(4)]:
                for o, got4 in fut.result():
                    check(got4, ("threads", o), slice(o, o + 4096))
    finally:
        for c in clones:
            c.close()


def test_api_edges_and_async(gv, coracle, golden):
    from pbft_amd import SigBatch, bitmap_to_bool
    b = dict(golden_batches(golden))[85]
    gv.set_keys(b["keys"])
    exp = b["expected"].astype(bool)
    for n in (1, 2, 63, 64, 65, 127, 200):
        got, bm = verify(gv, b["R"][:n], b["S"][:n], b["key_idx"][:n], b["msg"][:n], 85)
        assert (got == exp[:n]).all(), n
        assert len(bm) == (n + 63) // 64
        if n % 64:
            assert int(bm[-1]) >> (n % 64) == 0
    empty = gv.verify(SigBatch(b["R"][:0], b["S"][:0], b["key_idx"][:0], b["msg"][:0], 85))
    assert len(empty) == 0
    # async: submit, poll until done, equals sync
    t = gv.submit(SigBatch(b["R"], b["S"], b["key_idx"], b["msg"], 85))
    out = None
    while out is None:
        out = gv.poll(t)
    assert (bitmap_to_bool(out, len(exp)) == exp).all()
    # odd message stride (envelope embedded in wider records, unaligned)
    n = len(exp)
    wide = np.zeros((n, 93), dtype=np.uint8)
    wide[:, 3:88] = b["msg"]
    got, _ = verify(gv, b["R"], b["S"], b["key_idx"], wide[:, 3:].copy(), 85)
    assert (got == exp).all()


def test_device_entry_point(gv, golden):
    import torch
    from pbft_amd import bitmap_to_bool
    b = dict(golden_batches(golden))[85]
    gv.set_keys(b["keys"])
    dev = torch.device("cuda", 0)
    n = len(b["R"])
    for stride in (85, 87, 128):
        buf = np.zeros(n * stride + 64, dtype=np.uint8)
        buf[: n * stride].reshape(n, stride)[:, :85] = b["msg"]
        dR = torch.from_numpy(b["R"].copy()).to(dev)
        dS = torch.from_numpy(b["S"].copy()).to(dev)
        dK = torch.from_numpy(b["key_idx"].view(np.int16).copy()).to(dev)
        dM = torch.from_numpy(buf).to(dev)
        dB = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
        st = torch.cuda.Stream(dev)
        torch.cuda.synchronize()
        assert gv.last_kernel_ms() == -1  # (timing events are off by default since r05)
        gv.set_option(gv.OPT_KERNEL_TIMING, 1)
        with torch.cuda.stream(st):
            gv.verify_device(dR.data_ptr(), dS.data_ptr(), dK.data_ptr(), dM.data_ptr(), 85, stride, n,
                             dB.data_ptr(), st.cuda_stream)
        st.synchronize()
        got = bitmap_to_bool(dB.cpu().numpy().view(np.uint64), n)
        assert (got == b["expected"].astype(bool)).all(), stride
        assert gv.last_kernel_ms() > 0
        # PBFT_OPT_KERNEL_TIMING = 0: no timing events around the launch (same bits, no kernel time)
        gv.set_option(gv.OPT_KERNEL_TIMING, 0)
        try:
            dB.zero_()
            gv.verify_device(dR.data_ptr(), dS.data_ptr(), dK.data_ptr(), dM.data_ptr(), 85, stride, n,
                             dB.data_ptr(), st.cuda_stream)
            st.synchronize()
            assert (bitmap_to_bool(dB.cpu().numpy().view(np.uint64), n) == b["expected"].astype(bool)).all()
            assert gv.last_kernel_ms() == -1
            # the host-buffer path (submit / wait) twice in a row: no stale HIP error from the missing events
            from pbft_amd import SigBatch
            for _ in range(2):
                bm = gv.verify(SigBatch(b["R"], b["S"], b["key_idx"], b["msg"], 85))
                assert (bitmap_to_bool(bm, n) == b["expected"].astype(bool)).all()
        finally:
            gv.set_option(gv.OPT_KERNEL_TIMING, 0)


def test_digests_match_hashlib(gv):
    rng = random.Random(5)
    items = [b"", b"abc", b"testOperation"] + [rng.randbytes(rng.choice([1, 55, 56, 63, 64, 65, 111, 112, 127, 128,
                                                                          129, 255, 256, 1000]))
                                                for _ in range(500)]
    b2 = gv.blake2b512(items)
    s2 = gv.sha256(items)
    for i, it in enumerate(items):
        assert b2[i].tobytes() == hashlib.blake2b(it, digest_size=64).digest(), (i, len(it))
        assert s2[i].tobytes() == hashlib.sha256(it).digest(), (i, len(it))
    # the reference README's request (README.md:42) digest, src/message.rs:209-212
    assert b2[2].tobytes().hex() == KAT["digest"]["blake2b512_hex"]


def test_ctx_clone_shares_tables_and_snapshots_keys(gv, golden):
    """pbft_verify_ctx_clone: a second stream on the same tables; the clone keeps the key set it was made with."""
    from pbft_amd import SigBatch, bitmap_to_bool
    bs = dict(golden_batches(golden))
    b85, b0 = bs[85], bs[0]
    gv.set_keys(b85["keys"])
    c = gv.clone()
    try:
        exp = b85["expected"].astype(bool)
        batch = SigBatch(b85["R"], b85["S"], b85["key_idx"], b85["msg"], 85)
        # both contexts in flight at once (two HIP streams), same answer
        t1, t2 = gv.submit(batch), c.submit(batch)
        o2, o1 = c.wait(t2), gv.wait(t1)
        assert (bitmap_to_bool(o1, len(exp)) == exp).all()
        assert (bitmap_to_bool(o2, len(exp)) == exp).all()
        # replacing the parent's key set leaves the clone's snapshot in place
        gv.set_keys(b0["keys"])
        got0, _ = verify(gv, b0["R"], b0["S"], b0["key_idx"], b0["msg"], 0)
        assert (got0 == b0["expected"].astype(bool)).all()
        got85 = bitmap_to_bool(c.verify(batch), len(exp))
        assert (got85 == exp).all()
    finally:
        c.close()


def test_wire_records_and_stream_end_to_end(gv, golden):
    """Zero-copy binary records and UviBytes/JSON frames -> SoA -> GPU, bit-exact with the SoA path."""
    from pbft_amd import SigBatch, bitmap_to_bool, wire
    b = dict(golden_batches(golden))[85]
    gv.set_keys(b["keys"])
    exp = b["expected"].astype(bool)
    rec = wire.records_pack(b["R"], b["S"], b["key_idx"], b["msg"], b["msg"].shape[1])
    got = bitmap_to_bool(gv.verify_records(rec), len(exp))
    assert (got == exp).all()
    # a replica round on the wire: GPU-signed Prepare/Commit votes of n = 7 replicas, JSON frames
    n_rep, n_seq = 7, 40
    seeds = seeds_for(n_rep, tag=77)
    digests = [hashlib.blake2b(b"op-%d" % s, digest_size=64).digest() for s in range(n_seq)]
    rows = [(k, s, r) for s in range(n_seq) for k in (1, 2) for r in range(n_rep)]
    env = np.stack([np.frombuffer(b"PBFT" + bytes([k]) + (3).to_bytes(8, "little") + s.to_bytes(8, "little") +
                                  digests[s], np.uint8) for k, s, r in rows])
    kidx = np.array([r for _, _, r in rows], np.uint16)
    R, S, pub = gv.sign(seeds, kidx, env, 85)
    gv.set_keys(pub)
    frames = []
    for i, (k, s, r) in enumerate(rows):
        sig = bytes(R[i]) + bytes(S[i])
        if i % 17 == 3:  # corrupted on the wire
            sig = sig[:40] + bytes([sig[40] ^ 4]) + sig[41:]
        frames.append(wire.encode_frame(wire.WireMsg(kind=k, view=3, seq=s, digest=digests[s], replica=r, sig=sig)))
    v = wire.decode_votes(b"".join(frames), n_replicas=n_rep)
    assert (v.status == 0).all() and len(v.R) == len(rows)
    assert (v.msg == env).all()
    got = bitmap_to_bool(gv.verify(SigBatch(v.R, v.S, v.key_idx, v.msg, 85)), len(rows))
    assert (got == np.array([i % 17 != 3 for i in range(len(rows))])).all()


def test_latency_mode_split_kernel_matches_single_lane(golden):
    """comb_latency_kernel (4 lanes per signature, batches < 2^16) and comb_kernel give identical bitmaps on every
    golden batch (every adversarial class, every message length)."""
    from pbft_amd import GpuBatchVerifier
    results = {}
    for mode, thr in (("split", 1_000_000_000), ("single", 0)):
        v = GpuBatchVerifier(0)
        v.set_option(v.OPT_SPLIT_BELOW, thr)
        try:
            for ml, b in golden_batches(golden):
                v.set_keys(b["keys"])
                got, _ = verify(v, b["R"], b["S"], b["key_idx"], b["msg"], ml)
                assert (got == b["expected"].astype(bool)).all(), (mode, ml)
                results[(mode, ml)] = got
        finally:
            v.close()


def test_verify_batch_multi_shards(gv, golden):
    """pbft_verify_batch_multi over 3 contexts (cloned on this GPU; distinct GPUs in a multi-GPU process):
    64-aligned shards, empty trailing shards for tiny N, bitmap identical to one context."""
    from pbft_amd import SigBatch, bitmap_to_bool, verify_multi
    b = dict(golden_batches(golden))[85]
    gv.set_keys(b["keys"])
    clones = [gv.clone(), gv.clone()]
    try:
        exp = b["expected"].astype(bool)
        for n in (1, 64, 65, 130, len(exp)):
            batch = SigBatch(b["R"][:n], b["S"][:n], b["key_idx"][:n], b["msg"][:n], 85)
            got = bitmap_to_bool(verify_multi([gv] + clones, batch), n)
            assert (got == exp[:n]).all(), n
    finally:
        for c in clones:
            c.close()


def test_device_launch_captured_in_hip_graph(gv, golden):
    """pbft_verify_reserve + pbft_verify_batch_device captured into a HIP graph (torch.cuda.CUDAGraph on ROCm)
    and replayed: the replays give the oracle's bitmap (inputs swapped in place between replays)."""
    import torch
    from pbft_amd import bitmap_to_bool
    b = dict(golden_batches(golden))[85]
    gv.set_keys(b["keys"])
    exp = b["expected"].astype(bool)
    n = len(exp)
    dev = torch.device("cuda", 0)
    dR, dS = torch.from_numpy(b["R"].copy()).to(dev), torch.from_numpy(b["S"].copy()).to(dev)
    dK = torch.from_numpy(b["key_idx"].astype(np.uint16).view(np.int16)).to(dev)
    mp = np.zeros(n * 85 + 64, np.uint8)
    mp[: n * 85] = b["msg"].reshape(-1)
    dM = torch.from_numpy(mp).to(dev)
    dB = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
    gv.reserve(n)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        gv.verify_device(dR.data_ptr(), dS.data_ptr(), dK.data_ptr(), dM.data_ptr(), 85, 85, n, dB.data_ptr(),
                         torch.cuda.current_stream().cuda_stream)
    for rep in range(3):
        dB.zero_()
        if rep == 2:  # new inputs in the same buffers: every signature's S flipped -> all rejected
            dS.copy_(torch.from_numpy(b["S"] ^ 1).to(dev))
        g.replay()
        torch.cuda.synchronize()
        got = bitmap_to_bool(dB.cpu().numpy().view(np.uint64), n)
        assert (got == (exp if rep < 2 else np.zeros(n, bool))).all(), rep


def test_config2_pipelined_window(gv, coracle):
    """BASELINE configs[1]: n = 4 replicas, 1,024 pipelined requests -> 8,192 Prepare + Commit signatures in one
    window batch (latency-mode kernel), 1 % adversarial, bit-exact with the C oracle; the same batch through the
    one-lane-per-signature kernels (PBFT_OPT_SPLIT_BELOW = 0) gives the same bits, with every finish width, with
    and without the finish's cross-lane product tree (its wave inversion, inv25519.h fe_invert_wave), compiled for
    one or two waves per SIMD, also on a ragged batch (partial last wave)."""
    from pbft_amd import GpuBatchVerifier
    seeds, pub, R, S, key_idx, msg = round_batch(gv, 4, 1024, tag=2)
    assert len(R) == 8192
    assert gv.set_keys(pub).all()
    rng = np.random.default_rng(2)
    R2, S2, K2, M2, idx = adversarial(rng, pub, R, S, key_idx, msg)
    got, _ = verify(gv, R2, S2, K2, M2, 85)
    exp = oracle_bits(coracle, pub, R2, S2, K2, M2, 85)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
    assert not got[idx].any() and got.sum() == len(R) - len(idx)
    # the latency kernel with 4 and with 8 lanes per signature (by size: 8 up to 8,192), full and ragged
    n3 = len(R2) - 1000 - 37
    try:
        for sp in (4, 8):
            gv.set_option(gv.OPT_LAT_SPLIT, sp)
            got3, _ = verify(gv, R2, S2, K2, M2, 85)
            assert (got3 == exp).all(), sp
            got3, _ = verify(gv, R2[:n3], S2[:n3], K2[:n3], M2[:n3], 85)
            assert (got3 == exp[:n3]).all(), (sp, n3)
    finally:
        gv.set_option(gv.OPT_LAT_SPLIT, 0)
    v1 = gv.clone()
    v1.set_option(v1.OPT_SPLIT_BELOW, 0)
    try:
        v1.set_keys(pub)
        n2 = len(R2) - 37
        for lv, waves in ((0, 1), (4, 1), (4, 2)):  # (4, 2): the tree finish compiled for 2 waves per SIMD
            v1.set_option(v1.OPT_FINISH_TREE, lv)
            v1.set_option(v1.OPT_FINISH_WAVES, waves)
            for fm in (1, 2, 4, 8, 16):
                v1.set_option(v1.OPT_FINISH_WIDTH, fm)
                got1, _ = verify(v1, R2, S2, K2, M2, 85)
                assert (got1 == exp).all(), (fm, lv, waves)
                got2, _ = verify(v1, R2[:n2], S2[:n2], K2[:n2], M2[:n2], 85)
                assert (got2 == exp[:n2]).all(), (fm, lv, waves, n2)
        with pytest.raises(Exception):               # the tree depth that is not compiled
            v1.set_option(v1.OPT_FINISH_TREE, 6)
        with pytest.raises(Exception):
            v1.set_option(v1.OPT_FINISH_WIDTH, 3)
    finally:
        v1.close()


@pytest.mark.parametrize("budget_mb,pa", [("5000", 14), ("1500", 16), ("40", 32)])
def test_smaller_key_plans(gv, coracle, golden, budget_mb, pa):
    """The 14-, 16- and 32-position key plans (PLA_BIG / PLA_MID / PLA_SMALL), chosen by pbft_verify_set_keys when the key set does
    not fit PBFT_KEY_TABLE_BUDGET_MB: golden corpus (latency kernel) and a config-#3 round (comb kernel) bit-exact."""
    v = gv.clone()
    v.set_option(v.OPT_KEY_TABLE_BUDGET_MB, int(budget_mb))
    try:
        for ml, b in golden_batches(golden):
            assert (v.set_keys(b["keys"]) == b["key_ok"].astype(bool)).all()
            assert v.positions()[1] == pa
            got, _ = verify(v, b["R"], b["S"], b["key_idx"], b["msg"], ml)
            assert (got == b["expected"].astype(bool)).all(), (pa, ml)
        seeds, pub, R, S, key_idx, msg = round_batch(gv, 16, 2048, tag=9)   # 2^16 signatures, 16 replicas
        assert v.set_keys(pub).all() and v.positions()[1] == pa
        rng = np.random.default_rng(9)
        R2, S2, K2, M2, idx = adversarial(rng, pub, R, S, key_idx, msg)
        got, _ = verify(v, R2, S2, K2, M2, 85)
        exp = oracle_bits(coracle, pub, R2, S2, K2, M2, 85)
        assert (got == exp).all(), (pa, np.nonzero(got != exp)[0][:10])
    finally:
        v.close()


def test_pipelined_device_rounds(gv, coracle):
    """pbft_verify_batch_device_pipelined: consecutive rounds with the comb on one stream and the finish on another
    (two workspace halves, the comb of round k+1 overlapping the finish of round k); every round's bitmap equals the
    oracle's, including a latency-mode batch in the middle and a ragged tail."""
    import torch
    from pbft_amd import bitmap_to_bool
    seeds, pub, R, S, key_idx, msg = round_batch(gv, 64, 1024, tag=21)    # 131,072 signatures
    assert gv.set_keys(pub).all()
    rng = np.random.default_rng(21)
    rounds = []
    for k in range(5):
        R2, S2, K2, M2, idx = adversarial(rng, pub, R, S, key_idx, msg, frac=0.002)
        n = (len(R), len(R) - 37, 4096, len(R), 70_001)[k]
        rounds.append((R2[:n], S2[:n], K2[:n], M2[:n]))
    dev = torch.device("cuda", 0)
    import bench
    dsets = [bench.to_device(torch, dev, *r) for r in rounds]
    a, b = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    exps = [oracle_bits(coracle, pub, r[0], r[1], r[2], r[3], 85) for r in rounds]
    torch.cuda.synchronize()
    for rep in range(2):
        for ds, r in zip(dsets, rounds):
            ds["B"].zero_()
        torch.cuda.synchronize()
        for ds, r in zip(dsets, rounds):
            gv.verify_device_pipelined(ds["R"].data_ptr(), ds["S"].data_ptr(), ds["K"].data_ptr(), ds["M"].data_ptr(),
                                       85, 85, len(r[0]), ds["B"].data_ptr(), a.cuda_stream, b.cuda_stream)
        torch.cuda.synchronize()
        for ds, r, exp in zip(dsets, rounds, exps):
            got = bitmap_to_bool(ds["B"].cpu().numpy().view(np.uint64), len(r[0]))
            assert (got == exp).all(), (rep, len(r[0]), np.nonzero(got != exp)[0][:8])
    with pytest.raises(Exception):
        gv.verify_device_pipelined(0, 0, 0, 0, 85, 85, 1, 0, a.cuda_stream, a.cuda_stream)  # same stream twice


def test_votes_form_matches_oracle_and_soa(gv, coracle):
    """pbft_verify_votes: each signature names its window envelope in a table of distinct envelopes (70 B per
    signature over PCIe instead of 151).  Bit-exact with the oracle on an adversarial round, an out-of-range envelope
    index is bit 0, and the chunked path (N > 2^18) and the latency-mode path give the SoA path's bits."""
    from pbft_amd import SigBatch, bitmap_to_bool
    seeds, pub, R, S, key_idx, msg = round_batch(gv, 64, 512, tag=31)     # 65,536 signatures
    assert gv.set_keys(pub).all()
    rng = np.random.default_rng(31)
    R2, S2, K2, M2, idx = adversarial(rng, pub, R, S, key_idx, msg)
    env, inv = np.unique(M2, axis=0, return_inverse=True)
    ei = inv.reshape(-1).astype(np.uint32)
    n = len(R2)
    got = bitmap_to_bool(gv.verify_votes(R2, S2, K2, ei, env), n)
    exp = oracle_bits(coracle, pub, R2, S2, K2, M2, 85)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:8]
    bad = ei.copy()
    bad[::997] = len(env) + 5
    got2 = bitmap_to_bool(gv.verify_votes(R2, S2, K2, bad, env), n)
    mask = np.ones(n, bool)
    mask[::997] = False
    assert not got2[~mask].any() and (got2[mask] == exp[mask]).all()
    for m in (4096, 1000):                                                # latency-mode kernel
        g3 = bitmap_to_bool(gv.verify_votes(R2[:m], S2[:m], K2[:m], ei[:m], env), m)
        assert (g3 == exp[:m]).all(), m
    # shuffled: every wave mixes envelopes, so block 2's schedule comes from the per-envelope table (votes form)
    # or per lane (SoA) instead of the scalar unit -- the same bits
    perm = rng.permutation(n)
    g6 = bitmap_to_bool(gv.verify_votes(R2[perm], S2[perm], K2[perm], ei[perm], env), n)
    assert (g6 == exp[perm]).all()
    g7 = bitmap_to_bool(gv.verify(SigBatch(R2[perm], S2[perm], K2[perm], M2[perm], 85)), n)
    assert (g7 == exp[perm]).all()
    # 2^19 + 3 signatures: chunked H2D path; equals the SoA host path on the same rows
    reps = (1 << 19) // n + 1
    RR, SS, KK, II = (np.concatenate([a] * reps)[: (1 << 19) + 3] for a in (R2, S2, K2, ei))
    MM = env[II]
    g4 = bitmap_to_bool(gv.verify_votes(RR, SS, KK, II, env), len(RR))
    g5 = bitmap_to_bool(gv.verify(SigBatch(RR, SS, KK, MM, 85)), len(RR))
    assert (g4 == g5).all() and (g4[:n] == exp).all()


def test_async_host_forms_pinned_staging(gv, coracle):
    """The non-blocking host-buffer forms: pbft_verify_batch_async and pbft_verify_votes_async
    copy pageable buffers into the context's pinned staging before returning (the caller may reuse them at once:
    they are overwritten here while the batch runs), DMA pinned buffers in place, and the zero-copy
    pbft_verify_votes_stage / _submit pair fills the staging directly.  All equal the oracle."""
    import torch
    from pbft_amd import SigBatch, bitmap_to_bool
    seeds, pub, R, S, key_idx, msg = round_batch(gv, 16, 2048, tag=41)   # 65,536 signatures
    assert gv.set_keys(pub).all()
    rng = np.random.default_rng(41)
    R, S, K, M, _ = adversarial(rng, pub, R, S, key_idx, msg)
    exp = oracle_bits(coracle, pub, R, S, K, M, 85)
    n = len(R)
    env, inv = np.unique(M, axis=0, return_inverse=True)
    ei = inv.reshape(-1).astype(np.uint32)
    # pageable, overwritten right after submit
    for form in ("batch", "votes"):
        Rc, Sc, Kc, Mc, Ic, Ec = R.copy(), S.copy(), K.copy(), M.copy(), ei.copy(), env.copy()
        t = gv.submit(SigBatch(Rc, Sc, Kc, Mc, 85)) if form == "batch" else gv.submit_votes(Rc, Sc, Kc, Ic, Ec)
        for a in (Rc, Sc, Mc, Ec):
            a[:] = 0x5A
        Kc[:] = 1
        Ic[:] = 0
        out = gv.wait(t)
        assert (bitmap_to_bool(out, n) == exp).all(), form
    # pinned caller buffers: DMA'd in place (kept alive until completion)
    pin = lambda a: torch.from_numpy(np.ascontiguousarray(a)).pin_memory().numpy()  # noqa: E731
    t = gv.submit_votes(pin(R), pin(S), pin(K), pin(ei), pin(env))
    out = None
    while out is None:
        out = gv.poll(t)
    assert (bitmap_to_bool(out, n) == exp).all()
    # zero-copy staging
    st = gv.stage_votes(n, len(env))
    st["sig"][:, :32] = R
    st["sig"][:, 32:] = S
    st["key_idx"][:] = K
    st["env_idx"][:] = ei
    st["envelopes"][:] = env
    t = gv.submit_staged(n, len(env))
    assert (bitmap_to_bool(gv.wait(t), n) == exp).all()
    # a submit without a matching stage is refused; one batch in flight per context
    from pbft_amd import PbftError
    with pytest.raises(PbftError):
        gv.submit_staged(n, len(env))
    t = gv.submit_votes(R, S, K, ei, env)
    with pytest.raises(PbftError):
        gv.submit_votes(R, S, K, ei, env)
    gv.wait(t)


def test_progressive_votes_submit(gv, coracle):
    """pbft_verify_votes_submit_begin / _rows + pbft_verify_poll_rows (what pbft_replica_flush_submit and
    _flush_poll use): the staging is launched chunk by chunk as it is filled, each chunk's bitmap words come back
    on their own; until the last rows are submitted the batch reads "running" and a blocking wait is refused.
    2^19 + 3 rows = chunks [0, 2^16), [2^16, 3 * 2^16), [3 * 2^16, 5 * 2^16), [5 * 2^16, 7 * 2^16),
    [7 * 2^16, 2^19 + 3) (the schedule of include/pbft_verify.h PBFT_VOTES_CHUNK_END: two small chunks at either
    end); every prefix reported done equals the oracle."""
    import ctypes
    from pbft_amd import PbftError, bitmap_to_bool
    seeds, pub, R, S, key_idx, msg = round_batch(gv, 16, 2048, tag=47)   # 65,536 signatures
    assert gv.set_keys(pub).all()
    rng = np.random.default_rng(47)
    R, S, K, M, _ = adversarial(rng, pub, R, S, key_idx, msg)
    exp = oracle_bits(coracle, pub, R, S, K, M, 85)
    env, inv = np.unique(M, axis=0, return_inverse=True)
    ei = inv.reshape(-1).astype(np.uint32)
    N = (1 << 19) + 3
    reps = N // len(R) + 1
    RR, SS, KK, II, EE = (np.concatenate([a] * reps)[:N] for a in (R, S, K, ei, exp))
    L, ctx = gv._lib, gv._ctx
    st = gv.stage_votes(N, len(env))
    st["envelopes"][:] = env
    out = np.zeros((N + 63) // 64, np.uint64)
    rows_done = ctypes.c_uint64()
    # the first chunk's rows only
    h = 1 << 18
    st["sig"][:h, :32], st["sig"][:h, 32:], st["key_idx"][:h], st["env_idx"][:h] = RR[:h], SS[:h], KK[:h], II[:h]
    assert L.pbft_verify_votes_submit_begin(ctx, N, len(env), out.ctypes.data) == 0
    ends = [1 << 16, 3 << 16, 5 << 16, 7 << 16, N]
    assert L.pbft_verify_votes_submit_rows(ctx, 1000) == 0                # no whole chunk yet
    assert L.pbft_verify_votes_submit_rows(ctx, h + 5) == 0               # chunks 0 and 1 (the filled rows' whole chunks)
    assert L.pbft_verify_poll(ctx) == 0
    with pytest.raises(PbftError):
        from pbft_amd._lib import check
        check(L.pbft_verify_wait(ctx))
    seen = 0
    while seen < ends[1]:
        assert L.pbft_verify_poll_rows(ctx, ctypes.byref(rows_done)) == 0
        assert rows_done.value in (0, ends[0], ends[1])
        seen = rows_done.value
    assert (bitmap_to_bool(out[: seen // 64], seen) == EE[:seen]).all()
    st["sig"][h:, :32], st["sig"][h:, 32:], st["key_idx"][h:], st["env_idx"][h:] = RR[h:], SS[h:], KK[h:], II[h:]
    assert L.pbft_verify_votes_submit_rows(ctx, N) == 0
    prev = seen
    while True:
        rc = L.pbft_verify_poll_rows(ctx, ctypes.byref(rows_done))
        assert rc in (0, 1) and rows_done.value >= prev
        prev = rows_done.value
        assert (bitmap_to_bool(out[: min(prev, N) // 64], min(prev, N) // 64 * 64) == EE[: min(prev, N) // 64 * 64]).all()
        if rc == 1:
            break
    assert prev >= N and (bitmap_to_bool(out, N) == EE).all()
    # a second, one-shot batch on the same context is unaffected (no chunk read-back)
    assert (bitmap_to_bool(gv.verify_votes(R, S, K, ei, env), len(R)) == exp).all()


@pytest.mark.parametrize("N", [1, 4095, 65536 + 77, (1 << 18) + 1, (1 << 19) + 4099])
def test_votes_submit_host_rows(gv, coracle, N):
    """pbft_verify_votes_submit_host (r05: the replica's row arena handed over as it is): staged rows and the
    envelope table in the caller's pinned memory (pbft_host_alloc), the whole batch launched at once -- the chunk
    schedule with its last chunk cut to 16k rows above 2^18 rows -- and completed progressively
    (pbft_verify_poll_rows: every reported prefix equals the oracle).  Ragged sizes from one row to 2^19 + 4099;
    every adversarial class; argument errors; the context serves an ordinary batch afterwards."""
    import ctypes
    from pbft_amd import bitmap_to_bool
    seeds, pub, R, S, key_idx, msg = round_batch(gv, 16, 2048, tag=53)   # 65,536 signatures
    assert gv.set_keys(pub).all()
    rng = np.random.default_rng(53)
    R, S, K, M, _ = adversarial(rng, pub, R, S, key_idx, msg)
    exp = oracle_bits(coracle, pub, R, S, K, M, 85)
    env, inv = np.unique(M, axis=0, return_inverse=True)
    ei = inv.reshape(-1).astype(np.uint32)
    reps = N // len(R) + 1
    RR, SS, KK, II, EE = (np.concatenate([a] * reps)[:N] for a in (R, S, K, ei, exp))
    L, ctx = gv._lib, gv._ctx
    hr, he = ctypes.c_void_p(), ctypes.c_void_p()
    assert L.pbft_host_alloc(ctx, 72 * N, ctypes.byref(hr)) == 0 and hr.value
    assert L.pbft_host_alloc(ctx, 85 * len(env) + 16, ctypes.byref(he)) == 0 and he.value
    try:
        rows = np.ctypeslib.as_array((ctypes.c_uint8 * (72 * N)).from_address(hr.value)).reshape(N, 72)
        envs = np.ctypeslib.as_array((ctypes.c_uint8 * (85 * len(env))).from_address(he.value)).reshape(-1, 85)
        rows[:, :32], rows[:, 32:64] = RR, SS
        rows[:, 64:68] = np.stack([KK.astype(np.uint16).view(np.uint8).reshape(N, 2)[:, 0],
                                   KK.astype(np.uint16).view(np.uint8).reshape(N, 2)[:, 1],
                                   np.zeros(N, np.uint8), np.zeros(N, np.uint8)], axis=1)
        rows[:, 68:72] = II.view(np.uint8).reshape(N, 4)
        envs[:] = env
        out = np.zeros((N + 63) // 64, np.uint64)
        # argument errors: nothing launched
        assert L.pbft_verify_votes_submit_host(ctx, hr, 0, he, len(env), out.ctypes.data) != 0
        assert L.pbft_verify_votes_submit_host(ctx, None, N, he, len(env), out.ctypes.data) != 0
        assert L.pbft_verify_votes_submit_host(ctx, hr, N, he, 0, out.ctypes.data) != 0
        assert L.pbft_verify_votes_submit_host(ctx, hr, N, he, len(env), out.ctypes.data) == 0
        assert L.pbft_verify_votes_submit_host(ctx, hr, N, he, len(env), out.ctypes.data) != 0   # busy
        rows_done = ctypes.c_uint64()
        prev = 0
        while True:
            rc = L.pbft_verify_poll_rows(ctx, ctypes.byref(rows_done))
            assert rc in (0, 1) and rows_done.value >= prev
            prev = rows_done.value
            k = min(prev, N) // 64 * 64
            assert (bitmap_to_bool(out[: k // 64], k) == EE[:k]).all()
            if rc == 1:
                break
        assert prev >= N and (bitmap_to_bool(out, N) == EE).all()
    finally:
        assert L.pbft_host_free(ctx, hr) == 0 and L.pbft_host_free(ctx, he) == 0
    assert (bitmap_to_bool(gv.verify_votes(R[:4096], S[:4096], K[:4096], ei[:4096], env), 4096) == exp[:4096]).all()


def test_votes_staged_and_pageable_chunks(gv, coracle):
    """The votes form's chunked H2D path (the only one since r06 removed the zero-copy option) on the staged path
    (pbft_verify_votes_stage / _submit) and the pageable path (copied into the staging first), at a multi-chunk size,
    one chunk, and latency-mode sizes: the oracle's bits."""
    from pbft_amd import bitmap_to_bool
    seeds, pub, R, S, key_idx, msg = round_batch(gv, 16, 2048, tag=53)   # 65,536 signatures
    assert gv.set_keys(pub).all()
    rng = np.random.default_rng(53)
    R, S, K, M, _ = adversarial(rng, pub, R, S, key_idx, msg)
    exp = oracle_bits(coracle, pub, R, S, K, M, 85)
    env, inv = np.unique(M, axis=0, return_inverse=True)
    ei = inv.reshape(-1).astype(np.uint32)
    big = (1 << 18) + 3 * (1 << 16) + 77                                  # chunks 2^16, 2^17, 2^18, rest
    reps = big // len(R) + 1
    RR, SS, KK, II, EE = (np.concatenate([a] * reps)[:big] for a in (R, S, K, ei, exp))
    for n in (big, 1 << 16, 4096, 777):
        st = gv.stage_votes(n, len(env))
        st["sig"][:, :32], st["sig"][:, 32:] = RR[:n], SS[:n]
        st["key_idx"][:], st["env_idx"][:], st["envelopes"][:] = KK[:n], II[:n], env
        got = bitmap_to_bool(gv.wait(gv.submit_staged(n, len(env))), n)
        assert (got == EE[:n]).all(), ("staged", n, np.nonzero(got != EE[:n])[0][:8])
        got = bitmap_to_bool(gv.verify_votes(RR[:n], SS[:n], KK[:n], II[:n], env), n)
        assert (got == EE[:n]).all(), ("pageable", n)


def test_multi_gpu_rccl_allgather_one_rank(gv, coracle):
    """pbft_multi_create / pbft_verify_batch_device_multi on the one GPU of this box: a
    1-rank RCCL communicator, the shard verified into its slice of the padded rank-major bitmap, then
    ncclAllGather.  (Unmeasured on 8 GPUs: the multi-rank layout is the same as bench.py's, gloo-tested.)"""
    import torch
    from pbft_amd import MultiGpu, bitmap_to_bool
    seeds, pub, R, S, key_idx, msg = round_batch(gv, 8, 160, tag=43)     # 2,560 signatures
    assert gv.set_keys(pub).all()
    rng = np.random.default_rng(43)
    R, S, K, M, _ = adversarial(rng, pub, R, S, key_idx, msg)
    exp = oracle_bits(coracle, pub, R, S, K, M, 85)
    n = len(R) - 5                                                        # ragged: not a multiple of 64
    dev = torch.device("cuda", 0)
    dR, dS = torch.from_numpy(R[:n].copy()).to(dev), torch.from_numpy(S[:n].copy()).to(dev)
    dK = torch.from_numpy(K[:n].view(np.int16).copy()).to(dev)
    mp = np.zeros(n * 85 + 64, np.uint8)
    mp[: n * 85] = M[:n].reshape(-1)
    dM = torch.from_numpy(mp).to(dev)
    wpr = (n + 63) // 64 + 3                                              # padded slice: 3 extra words
    dB = torch.full((wpr,), -1, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    m = MultiGpu([gv])
    try:
        m.verify_device([dR.data_ptr()], [dS.data_ptr()], [dK.data_ptr()], [dM.data_ptr()], [n], wpr,
                        [dB.data_ptr()])
        m.sync()
    finally:
        m.close()
    words = dB.cpu().numpy().view(np.uint64)
    assert (bitmap_to_bool(words, n) == exp[:n]).all()
    assert (words[(n + 63) // 64:] == 0).all()                            # padding words zeroed
    assert int(words[n // 64]) >> (n % 64) == 0                          # bits past n


def test_rekey_in_place_and_partial_update(gv, coracle):
    """a re-key with the same plan reuses the table allocation (no hipFree / hipMalloc), a
    smaller set too; pbft_verify_update_keys rebuilds only the named keys' tables -- a round signed under the
    updated set equals the oracle's bitmap over that set, the replaced keys' old signatures now fail, a
    small-order replacement key rejects everything under it; plan changes rebuild in place while the tables fit
    the allocation, a larger set re-allocates."""
    from pbft_amd import GpuBatchVerifier, PbftError
    seeds, pub, R, S, key_idx, msg = round_batch(gv, 64, 256, tag=31)   # 32,768 signatures
    rng = np.random.default_rng(31)
    R2, S2, K2, M2, _ = adversarial(rng, pub, R, S, key_idx, msg, frac=0.01)
    assert gv.set_keys(pub).all()
    assert gv.set_keys(pub).all()
    st = gv.key_stats()
    assert st["reused"] == 1 and st["free_ms"] == 0 and st["alloc_ms"] == 0 and st["keys_built"] == 64
    got, _ = verify(gv, R2, S2, K2, M2, 85)
    assert (got == oracle_bits(coracle, pub, R2, S2, K2, M2, 85)).all()
    # a smaller set in the same allocation: key indices >= 48 are out of the set (bit 0)
    assert gv.set_keys(pub[:48]).all() and gv.key_stats()["reused"] == 1
    got, _ = verify(gv, R2, S2, K2, M2, 85)
    exp = oracle_bits(coracle, np.ascontiguousarray(pub[:48]), R2, S2, K2, M2, 85)
    assert (got == exp).all() and not got[key_idx >= 48].any()
    assert gv.set_keys(pub).all() and gv.key_stats()["reused"] == 1
    # replace replicas 5 and 40 (new identities); the round re-signed under the new set
    slots = np.array([5, 40], np.uint32)
    seeds_new = seeds.copy()
    seeds_new[slots] = seeds_for(2, tag=32)
    Rn, Sn, pub_new = gv.sign(seeds_new, key_idx, msg, 85)
    assert (pub_new[np.setdiff1d(np.arange(64), slots)] == pub[np.setdiff1d(np.arange(64), slots)]).all()
    assert gv.update_keys(slots, pub_new[slots]).all()
    st = gv.key_stats()
    assert st["keys_built"] == 2 and st["reused"] == 1
    Rn2, Sn2, Kn2, Mn2, _ = adversarial(rng, pub_new, Rn, Sn, key_idx, msg, frac=0.01)
    got, _ = verify(gv, Rn2, Sn2, Kn2, Mn2, 85)
    assert (got == oracle_bits(coracle, pub_new, Rn2, Sn2, Kn2, Mn2, 85)).all()
    old, _ = verify(gv, R, S, key_idx, msg, 85)
    replaced = np.isin(key_idx, slots)
    assert not old[replaced].any() and old[~replaced].all()
    # a small-order replacement: key_ok 0, every signature under it rejects
    so = np.frombuffer(bytes.fromhex(KAT["small_order_encodings"][0]), np.uint8).reshape(1, 32)
    assert not gv.update_keys([7], so).any()
    got, _ = verify(gv, Rn, Sn, key_idx, msg, 85)
    assert not got[key_idx == 7].any() and got[(key_idx != 7)].all()
    for bad in ([64], [3, 3]):
        with pytest.raises(PbftError) as e:
            gv.update_keys(bad, pub_new[: len(bad)])
        assert e.value.code == -1
    # a plan change to smaller tables (budget forced down) rebuilds in the same allocation, and so does the
    # change back (the allocation never shrinks)
    pa0 = gv.positions()[1]
    gv.set_option(gv.OPT_KEY_TABLE_BUDGET_MB, 5000)   # 64 keys x 63 MB: the 16-position plan
    try:
        assert gv.set_keys(pub_new).all() and gv.positions()[1] == 16 and gv.key_stats()["reused"] == 1
        got, _ = verify(gv, Rn2, Sn2, Kn2, Mn2, 85)
        assert (got == oracle_bits(coracle, pub_new, Rn2, Sn2, Kn2, Mn2, 85)).all()
    finally:
        gv.set_option(gv.OPT_KEY_TABLE_BUDGET_MB, 0)
    assert gv.set_keys(pub_new).all() and gv.positions()[1] == pa0 and gv.key_stats()["reused"] == 1
    got, _ = verify(gv, Rn2, Sn2, Kn2, Mn2, 85)
    assert (got == oracle_bits(coracle, pub_new, Rn2, Sn2, Kn2, Mn2, 85)).all()
    # a set larger than the allocation frees and re-allocates (a fresh context: 8 keys, then 64, then 8 again)
    v2 = GpuBatchVerifier(0)
    try:
        assert v2.set_keys(pub_new[:8]).all() and v2.key_stats()["reused"] == 0
        assert v2.set_keys(pub_new).all() and v2.key_stats()["reused"] == 0
        got, _ = verify(v2, Rn2, Sn2, Kn2, Mn2, 85)
        assert (got == oracle_bits(coracle, pub_new, Rn2, Sn2, Kn2, Mn2, 85)).all()
        assert v2.set_keys(pub_new[:8]).all() and v2.key_stats()["reused"] == 1
    finally:
        v2.close()


def test_update_keys_failure_keeps_shared_set_consistent(gv, coracle):
    """pbft_verify_update_keys failing before anything is written (PBFT_OPT_FAULT_INJECT 1, as
    if its scratch allocation failed) leaves the key set -- shared with a clone -- unchanged; failing after the
    updated keys' tables were written (2) clears their key_ok in the shared set, so both contexts reject signatures
    under those slots and keep verifying every other key; a later successful update restores the slots."""
    from pbft_amd import PbftError
    seeds, pub, R, S, key_idx, msg = round_batch(gv, 16, 64, tag=61)      # 2,048 signatures
    assert gv.set_keys(pub).all()
    cl = gv.clone()
    try:
        slots = np.array([3, 9], np.uint32)
        seeds_new = seeds.copy()
        seeds_new[slots] = seeds_for(2, tag=62)
        Rn, Sn, pub_new = gv.sign(seeds_new, key_idx, msg, 85)
        hit = np.isin(key_idx, slots)
        gv.set_option(gv.OPT_FAULT_INJECT, 1)
        with pytest.raises(PbftError):
            gv.update_keys(slots, pub_new[slots])
        for v in (gv, cl):
            got, _ = verify(v, R, S, key_idx, msg, 85)
            assert got.all()                                              # unchanged, on both contexts
        gv.set_option(gv.OPT_FAULT_INJECT, 2)
        with pytest.raises(PbftError):
            gv.update_keys(slots, pub_new[slots])
        for v in (gv, cl):
            got, _ = verify(v, R, S, key_idx, msg, 85)
            assert not got[hit].any() and got[~hit].all()
            got, _ = verify(v, Rn, Sn, key_idx, msg, 85)
            assert not got[hit].any() and got[~hit].all()
        assert gv.update_keys(slots, pub_new[slots]).all()                 # the injection was one-shot
        for v in (gv, cl):
            got, _ = verify(v, Rn, Sn, key_idx, msg, 85)
            assert got.all()
            assert (got == oracle_bits(coracle, pub_new, Rn, Sn, key_idx, msg, 85)).all()
        with pytest.raises(PbftError):
            gv.set_option(gv.OPT_FAULT_INJECT, 3)
    finally:
        cl.close()
