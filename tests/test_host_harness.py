"""The product's __host__ __device__ arithmetic compiled for the host (tests/native/host_harness.cpp).

These run without a GPU: the exact field / SHA-512 / Barrett / decompress /
comb-table / verify_lane code that the HIP kernels execute is checked against
the oracle, so arithmetic bugs are caught before a GPU run.  The GPU tests
(test_gpu_*.py) then check the compiled gfx950 kernels bit-exactly.
"""
import ctypes
import hashlib
import os
import random

import numpy as np
import pytest

import ed25519_ref as E
from conftest import ROOT, golden_batches

P = E.P


@pytest.fixture(scope="module")
def hh():
    path = os.path.join(ROOT, "tests", "native", "libhost_harness.so")
    if not os.path.exists(path):
        pytest.skip("host harness not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    lib.hh_build_table.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int, vp]
    lib.hh_verify_batch.argtypes = [ctypes.c_int, vp, vp, vp, vp, ctypes.c_uint32, vp, vp, vp, vp, ctypes.c_uint32,
                                    ctypes.c_uint32, ctypes.c_uint64, vp]
    lib.hh_comb2.argtypes = [ctypes.c_int, vp, vp, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
    return lib


def _fe(hh, op, a, b):
    out = ctypes.create_string_buffer(32)
    hh.hh_fe_op(op, a.to_bytes(32, "little"), b.to_bytes(32, "little"), out)
    return int.from_bytes(out.raw, "little")


def test_field_ops(hh):
    rnd = random.Random(7)
    edge = [0, 1, 2, 18, 19, P - 1, P, P + 1, P + 18, 2**255 - 1, 2**255 - 2, 2**254, 2**26 - 1, 2**51]
    vals = edge + [rnd.randrange(2**255) for _ in range(600)]
    for i, a in enumerate(vals):
        b = vals[(i * 7 + 3) % len(vals)]
        assert _fe(hh, 0, a, b) == a * b % P
        assert _fe(hh, 1, a, b) == a * a % P
        assert _fe(hh, 4, a, b) == (a + b) ** 2 % P
        assert _fe(hh, 5, a, b) == (a - b) * b % P
        assert _fe(hh, 6, a, b) == (a + b) ** 2 % P
        # latency-oriented (parallel-carry) reductions: same values
        assert _fe(hh, 7, a, b) == a * b % P
        assert _fe(hh, 8, a, b) == a * a % P
        assert _fe(hh, 11, a, b) == (a + b) ** 2 % P
        assert _fe(hh, 12, a, b) == (a - b) * b % P
        assert _fe(hh, 13, a, b) == (b - a * a) * (a * a) % P
    for a in vals:
        assert _fe(hh, 14, a, 0) == pow(a, P - 2, P), a                  # divsteps inversion
    for i, a in enumerate(vals[:200]):
        b = vals[(i * 5 + 1) % len(vals)]
        assert _fe(hh, 15, a, b) == pow(a + b, P - 2, P)
    for a in vals[:60]:
        assert _fe(hh, 2, a, 0) == pow(a, P - 2, P)
        assert _fe(hh, 3, a, 0) == pow(a, (P - 5) // 8, P)
        assert _fe(hh, 9, a, 0) == pow(a, P - 2, P)
        assert _fe(hh, 10, a, 0) == pow(a, (P - 5) // 8, P)


def test_divsteps_inversion_extremes(hh):
    """safegcd inversion (pbft_amd/csrc/inv25519.h), constant- and variable-time, on inputs that stress the divstep
    count and the limb ranges:
    powers of two, p - 2^k, all-ones patterns, values just below p and unreduced encodings >= p."""
    vals = [2**k for k in range(255)] + [P - 2**k for k in range(1, 255)] + [(2**k - 1) for k in range(1, 256)]
    vals += [P - k for k in range(1, 40)] + [P + k for k in range(0, 19)] + [2**255 - 1 - k for k in range(20)]
    rnd = random.Random(99)
    vals += [rnd.getrandbits(rnd.randrange(1, 256)) for _ in range(2000)]
    for a in vals:
        assert _fe(hh, 14, a % 2**255, 0) == pow(a % 2**255, P - 2, P), a
        assert _fe(hh, 16, a % 2**255, 0) == pow(a % 2**255, P - 2, P), a  # variable-time form (finish tree)
    for i, a in enumerate(vals[:300]):
        b = vals[(i * 7 + 3) % len(vals)] % 2**255
        assert _fe(hh, 17, a % 2**255, b) == pow(a % 2**255 + b, P - 2, P)


def test_table_divsteps_match_divsteps30(hh):
    """divsteps30_tab (6 lookups of 5 half-delta divsteps in the 5,120-entry table, inv25519.h) returns the same
    transition matrix and zeta as the step-by-step divsteps30, zeta classes on both sides of the clamp included."""
    hh.hh_divsteps_tab_check.restype = ctypes.c_int
    assert hh.hh_divsteps_tab_check(ctypes.c_uint64(0x9E3779B97F4A7C15), 300000) == 0


def test_wave_inversion_emulation(hh):
    """fe_invert_tab and the lane-parallel fe_invert_wave (its host emulation: 16-lane rows, DPP shifts and
    readlanes spelled out, every limb bound asserted) equal z^(p-2) on the inversion extremes and random values."""
    vals = [2**k for k in range(255)] + [P - 2**k for k in range(1, 255)] + [(2**k - 1) for k in range(1, 256)]
    vals += [P - k for k in range(1, 40)] + [P + k for k in range(0, 19)] + [2**255 - 1 - k for k in range(20)] + [0]
    rnd = random.Random(1234)
    vals += [rnd.getrandbits(rnd.randrange(1, 256)) for _ in range(1500)]
    for a in vals:
        want = pow(a % 2**255, P - 2, P)
        assert _fe(hh, 18, a % 2**255, 0) == want, a
        assert _fe(hh, 20, a % 2**255, 0) == want, a   # (a bound violation would return 1000 + its site)
    for i, a in enumerate(vals[:300]):
        b = vals[(i * 7 + 3) % len(vals)] % 2**255
        assert _fe(hh, 19, a % 2**255, b) == pow(a % 2**255 + b, P - 2, P)
        assert _fe(hh, 21, a % 2**255, b) == pow(a % 2**255 + b, P - 2, P)


@pytest.mark.parametrize("ln", [0, 1, 47, 48, 63, 64, 85, 111, 112, 175, 176, 239, 240, 300, 1023])
def test_sha512_ram(hh, ln):
    rnd = random.Random(ln)
    r, a, m = rnd.randbytes(32), rnd.randbytes(32), rnd.randbytes(ln)
    buf = m + bytes(16)
    out = ctypes.create_string_buffer(64)
    for fixed in (0, 1):  # runtime length, and the compile-time specialisation (padding folded, last block peeled)
        hh.hh_sha512_ram(r, a, buf, ln, out, fixed)
        assert out.raw == hashlib.sha512(r + a + m).digest(), fixed


def test_sha512_ram_envelope_schedule(hh):
    """Votes form: the 85-byte envelope's block-2 schedule computed once (sha512_env_sched) and the per-signature
    hash that reads it (sha512_ram_env), and sha512_ram85's per-lane path, give SHA-512(R || A || M) (the
    wave-uniform scalar path is device-only: the GPU round tests cover it)."""
    rnd = random.Random(85)
    out = ctypes.create_string_buffer(64)
    for k in range(300):
        r, a, m = rnd.randbytes(32), rnd.randbytes(32), rnd.randbytes(85)
        if k < 4:
            m = bytes([[0x00, 0xFF, 0x80, 0x7F][k]]) * 85
        hh.hh_sha512_ram_env(r, a, m + bytes(16), out)
        assert out.raw == hashlib.sha512(r + a + m).digest(), k
        hh.hh_sha512_ram85(r, a, m + bytes(16), out)
        assert out.raw == hashlib.sha512(r + a + m).digest(), k


def test_reduce512(hh):
    rnd = random.Random(11)
    L = E.L
    vals = [0, 1, L - 1, L, L + 1, 2 * L, 3 * L - 1, 2**512 - 1, 2**256, 2**253] + [rnd.randrange(2**512)
                                                                                     for _ in range(3000)]
    # the radix-2^21 fold (sc_reduce512_fold): multiples of L and of 2^252 +- small, limbs all ones / zero,
    # values whose folds cancel (the result lands just below 0 or just above L before the final +L)
    vals += [k * L + r for k in (1, 2**7, 2**100, 2**259 - 1) for r in (0, 1, L - 1) if k * L + r < 2**512]
    vals += [j * 2**252 + r for j in (1, 2, 2**259 - 1) for r in (0, 1, 2**252 - 1)]
    vals += [(2**(21 * i) - 1) for i in range(1, 25)] + [2**512 - 2**(21 * i) for i in range(1, 25)]
    vals += [rnd.randrange(2**252) * L % 2**512 for _ in range(200)]
    for x in vals:
        out = ctypes.create_string_buffer(32)
        hh.hh_reduce512(x.to_bytes(64, "little"), out)
        assert int.from_bytes(out.raw, "little") == x % L


def test_decompress(hh, golden):
    rnd = random.Random(5)
    import json
    kat = json.load(open(os.path.join(ROOT, "tests", "golden", "kat.json")))
    encs = [bytes.fromhex(h) for h in kat["small_order_encodings"] + kat["noncanonical_decodable_encodings"]]
    encs += [rnd.randbytes(32) for _ in range(300)] + [E.compress(E.BASE)]
    for enc in encs:
        out = ctypes.create_string_buffer(32)
        rc = hh.hh_decompress(enc, out)
        p = E.decompress(enc)
        if p is None:
            assert rc == 0
        else:
            assert rc == (2 if E.is_small_order(p) else 1)
            assert out.raw == E.compress(p)


def test_comb_tables_and_mul(hh):
    tb = np.zeros(hh.hh_table_words(4), dtype=np.uint32)
    ta = np.zeros_like(tb)
    assert hh.hh_build_table(4, E.compress(E.BASE), 0, tb.ctypes.data) == 1
    A = E.pt_mul(987654321, E.BASE)
    assert hh.hh_build_table(4, E.compress(A), 1, ta.ctypes.data) == 1
    rnd = random.Random(9)
    out = ctypes.create_string_buffer(32)
    cases = [(0, 0), (1, 0), (0, 1), (8, 0), (0x88, 0x99), (E.L - 1, E.L - 1), (2**252, 3)]
    cases += [(rnd.randrange(E.L), rnd.randrange(E.L)) for _ in range(20)]
    for s, k in cases:
        hh.hh_comb2(4, tb.ctypes.data, ta.ctypes.data, s.to_bytes(32, "little"), k.to_bytes(32, "little"), out)
        assert out.raw == E.compress(E.pt_add(E.pt_mul(s, E.BASE), E.pt_mul(k, E.pt_neg(A)))), (s, k)


@pytest.mark.parametrize("W", [4, 67])  # 67: the non-uniform plan<40, 6, 14> (balanced 7/6-bit windows)
def test_verify_lane_golden(hh, golden, W):
    tw = hh.hh_table_words(W)
    tabB = np.zeros(tw, dtype=np.uint32)
    assert hh.hh_build_table(W, E.compress(E.BASE), 0, tabB.ctypes.data) == 1
    for ml, b in golden_batches(golden):
        keys, kok = b["keys"], b["key_ok"]
        tabA = np.zeros((len(keys), tw), dtype=np.uint32)
        for i in range(len(keys)):
            hh.hh_build_table(W, keys[i].tobytes(), 1, tabA[i].ctypes.data)
        n, stride = len(b["R"]), b["msg"].shape[1]
        mbuf = np.zeros(n * stride + 16, dtype=np.uint8)
        mbuf[: n * stride] = b["msg"].ravel()
        acc = np.zeros(n, dtype=np.uint8)
        assert hh.hh_verify_batch(W, tabB.ctypes.data, tabA.ctypes.data, keys.ctypes.data, kok.ctypes.data, len(keys),
                                  b["R"].ctypes.data, b["S"].ctypes.data, b["key_idx"].ctypes.data, mbuf.ctypes.data,
                                  ml, stride, n, acc.ctypes.data) == 0
        assert (acc == b["expected"]).all(), (ml, np.nonzero(acc != b["expected"])[0][:10])


_GUARD_SCRIPT = r"""
import ctypes, sys
import numpy as np
sys.path.insert(0, {tests!r})
from conftest import golden_batches
lib = ctypes.CDLL({lib!r})
vp = ctypes.c_void_p
lib.hh_guard_verify.argtypes = [ctypes.c_char_p, vp, vp, vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, vp,
                                ctypes.c_int]
g = np.load({npz!r})
b = dict(golden_batches(g))[85]
probe = {probe}
sel = np.nonzero((b["key_idx"] == 0) & np.isin(b["cls"], [0, 3, 4, 5, 17, 19]))[0]
if probe:
    sel = sel[b["cls"][sel] == 19]
R, S = np.ascontiguousarray(b["R"][sel]), np.ascontiguousarray(b["S"][sel])
if probe:
    S[:] = 0xff  # s = 2^256 - 1
M = np.zeros(len(sel) * 85 + 16, np.uint8)
M[: len(sel) * 85] = b["msg"][sel].ravel()
acc = np.zeros(len(sel), np.uint8)
rc = lib.hh_guard_verify(b["keys"][0].tobytes(), R.ctypes.data, S.ctypes.data, M.ctypes.data, 85, 85, len(sel),
                         acc.ctypes.data, probe)
assert rc == 0, rc
if not probe:
    assert (acc == b["expected"][sel]).all()
    assert (b["cls"][sel] == 19).sum() >= 1
print("ok", len(sel))
"""


def _guard_run(probe: int):
    import subprocess
    import sys
    lib = os.path.join(ROOT, "tests", "native", "libhost_harness.so")
    if not os.path.exists(lib):
        pytest.skip("host harness not built")
    code = _GUARD_SCRIPT.format(tests=os.path.join(ROOT, "tests"), lib=lib,
                                npz=os.path.join(ROOT, "tests", "golden", "verify_vectors.npz"), probe=probe)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)


def test_guard_page_no_gather_past_tables():
    """both comb tables end at a PROT_NONE page; the product's verify_lane on golden lanes incl.
    class 19 (s with bits 253..255 set) reads nothing past either table and gives the oracle's bits."""
    p = _guard_run(0)
    assert p.returncode == 0 and p.stdout.startswith("ok"), (p.returncode, p.stdout, p.stderr[-2000:])


def test_guard_page_catches_unclamped_recoding():
    """Negative control: recoding s = 2^256 - 1 WITHOUT the s < L clamp (the r01 kernels) faults on the guard page,
    so the test above would have caught the defect."""
    p = _guard_run(1)
    assert p.returncode == -11, (p.returncode, p.stdout, p.stderr[-2000:])
