#!/usr/bin/env python3
"""Generate the committed golden fixtures for the Ed25519 batch-verify hot path.

TEST INFRASTRUCTURE.  Run from the repo root:  python tests/golden/gen_golden.py

Expected outputs come from the pure-Python restatement oracle/ed25519_ref.py
(ed25519-dalek 1.0.1 verify_strict semantics; see its header for the crate
citations).  The reference repository has no tests and no signatures on its
messages (src/behavior.rs:127, :185), so these vectors are the build's own
artefacts; they are pinned by the RFC 8032 KATs in kat.json and cross-checked
against the C oracle and libsodium/OpenSSL in tests/test_oracle.py.

Outputs (all data, no code):
  tests/golden/kat.json            RFC 8032 / RFC 7693 / digest known answers
  tests/golden/verify_vectors.npz  SoA batches, one per message length, with
                                   expected accept bytes and a class id per lane
"""
from __future__ import annotations

import hashlib
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ed25519_ref as E  # noqa: E402

SEED = 0x5EED0000

CLASSES = {
    0: "valid",
    1: "message bit-flip",
    2: "R bit-flip",
    3: "s bit-flip",
    4: "s + L (non-canonical s)",
    5: "s with bit 255 set",
    6: "R not on curve",
    7: "R non-canonical y+p encoding",
    8: "R small-order encoding",
    9: "A small-order key",
    10: "A mixed-order key, equation-valid (accept)",
    11: "wrong key index",
    12: "all-zero signature",
    13: "R with torsion, cofactored-only valid (reject)",
    14: "A mixed-order key, cofactored-only valid (reject)",
    15: "A non-canonical y+p key",
    16: "A not on curve",
    17: "s = 0 / s = L-1 random R",
    18: "valid, s high nibble set (s >= 2^252)",
    19: "s >= 2^253 (bits 253-255: 2^256-1, s + 2^253, s | 2^254)",
}


def key_seed(i: int, seed: int = SEED) -> bytes:
    """sk_i = SHA-512("pbft-key" || seed || i)[0:32]."""
    return hashlib.sha512(b"pbft-key" + seed.to_bytes(8, "little") + i.to_bytes(8, "little")).digest()[:32]


def envelope(kind: int, view: int, seq: int) -> bytes:
    """85-byte signed envelope: "PBFT" || kind u8 || view u64 LE || seq u64 LE || digest[64]."""
    d = E.request_digest(b"op-" + str(seq).encode())
    return b"PBFT" + bytes([kind]) + view.to_bytes(8, "little") + seq.to_bytes(8, "little") + d


def enc_int(y: int, sign: int = 0) -> bytes:
    return (y | (sign << 255)).to_bytes(32, "little")


def torsion8():
    """A point of exact order 8: [L]Q for a curve point Q with a full torsion component."""
    y = 2
    while True:
        q = E.decompress(enc_int(y))
        if q is not None:
            t = E.pt_mul(E.L, q)
            t4 = E.pt_mul(4, t)
            if not E.is_identity(t4):
                return t
        y += 1


T8 = torsion8()
TORSION = [E.pt_mul(j, T8) for j in range(8)]


def small_order_encodings():
    out = set()
    for t in TORSION:
        out.add(E.compress(t))
    # x = 0 points (y = 1, y = -1) with the sign bit set: decompress accepts them
    out.add(enc_int(1, 1))
    out.add(enc_int(E.P - 1, 1))
    # non-canonical y + p encodings of y = 0 and y = 1
    for yv in (E.P, E.P + 1):
        for s in (0, 1):
            out.add(enc_int(yv, s))
    encs = sorted(out)
    for b in encs:
        p = E.decompress(b)
        assert p is not None and E.is_small_order(p), b.hex()
    return encs


SMALL_ORDER = small_order_encodings()
NONCANON = [enc_int(E.P + t, s) for t in range(19) for s in (0, 1)
            if E.decompress(enc_int(E.P + t, s)) is not None]


def not_on_curve(rnd: random.Random) -> bytes:
    while True:
        b = bytearray(rnd.randbytes(32))
        b[31] &= 0x7F
        if int.from_bytes(b, "little") >= E.P:
            continue
        if E.decompress(bytes(b)) is None:
            b[31] |= rnd.randrange(2) << 7
            return bytes(b)


def secret_scalar(seed: bytes) -> int:
    return E.secret_expand(seed)[0]


def mixed_key(seed: bytes, j: int = 1):
    a = secret_scalar(seed)
    A = E.pt_add(E.pt_mul(a, E.BASE), TORSION[j])
    return a, A, E.compress(A)


def sign_mixed(a: int, A_bytes: bytes, T_A_index: int, msg: bytes, rnd: random.Random) -> bytes:
    """Equation-valid signature under A = aB + T_A: needs R's torsion = -k*T_A."""
    while True:
        r = rnd.randrange(1, E.L)
        for j in range(8):
            R = E.pt_add(E.pt_mul(r, E.BASE), TORSION[j])
            rb = E.compress(R)
            k = E.scalar_from_hash(E.sha512(rb + A_bytes + msg))
            if (-(k * T_A_index)) % 8 == j:
                s = (r + k * a) % E.L
                return rb + s.to_bytes(32, "little")


def sign_cofactored_only(a: int, A_bytes: bytes, msg: bytes, rnd: random.Random, T_A_index: int = 0) -> bytes:
    """R = rB + T with the wrong torsion: [8](sB - kA - R) = O but sB - kA != R."""
    while True:
        r = rnd.randrange(1, E.L)
        j = rnd.randrange(1, 8)
        R = E.pt_add(E.pt_mul(r, E.BASE), TORSION[j])
        rb = E.compress(R)
        k = E.scalar_from_hash(E.sha512(rb + A_bytes + msg))
        if (-(k * T_A_index)) % 8 != j:
            s = (r + k * a) % E.L
            return rb + s.to_bytes(32, "little")


def build_batch(rnd: random.Random, msg_len: int, n_valid: int, n_each_adv: int):
    """One SoA batch with a shared message length; returns dict of arrays."""
    keys = []     # 32-byte encodings in the batch key table
    seeds = {}    # key index -> seed (for normal keys)
    n_norm = 8
    for i in range(n_norm):
        s = key_seed(i)
        seeds[i] = s
        keys.append(E.public_key(s))
    # special keys
    so_key = len(keys); keys.append(SMALL_ORDER[rnd.randrange(len(SMALL_ORDER))])
    mixed_j = 3
    mseed = key_seed(100)
    ma, _, mbytes = mixed_key(mseed, mixed_j)
    mixed_key_idx = len(keys); keys.append(mbytes)
    nc_key = len(keys); keys.append(NONCANON[rnd.randrange(len(NONCANON))])
    noc_key = len(keys); keys.append(not_on_curve(rnd))

    def rmsg():
        if msg_len == 85:
            return envelope(rnd.choice((1, 2)), 1, rnd.randrange(1, 1 << 20))
        return rnd.randbytes(msg_len)

    R, S, KI, M, CLS = [], [], [], [], []

    def add(sig: bytes, ki: int, m: bytes, cls: int):
        R.append(sig[:32]); S.append(sig[32:]); KI.append(ki); M.append(m); CLS.append(cls)

    def valid_sig(ki=None):
        ki = rnd.randrange(n_norm) if ki is None else ki
        m = rmsg()
        return E.sign(seeds[ki], m), ki, m

    for _ in range(n_valid):
        sig, ki, m = valid_sig()
        add(sig, ki, m, 0 if sig[63] & 0xF0 == 0 else 18)
    for _ in range(n_each_adv):
        sig, ki, m = valid_sig()
        if msg_len > 0:
            mm = bytearray(m); bi = rnd.randrange(8 * msg_len); mm[bi // 8] ^= 1 << (bi % 8)
            add(sig, ki, bytes(mm), 1)
        sig, ki, m = valid_sig()
        ss = bytearray(sig); bi = rnd.randrange(256); ss[bi // 8] ^= 1 << (bi % 8)
        add(bytes(ss), ki, m, 2)
        sig, ki, m = valid_sig()
        ss = bytearray(sig); bi = rnd.randrange(250); ss[32 + bi // 8] ^= 1 << (bi % 8)
        add(bytes(ss), ki, m, 3)
        sig, ki, m = valid_sig()
        s = int.from_bytes(sig[32:], "little") + E.L
        add(sig[:32] + s.to_bytes(32, "little"), ki, m, 4)
        sig, ki, m = valid_sig()
        s = int.from_bytes(sig[32:], "little") | (1 << 255)
        add(sig[:32] + s.to_bytes(32, "little"), ki, m, 5)
        sig, ki, m = valid_sig()
        add(not_on_curve(rnd) + sig[32:], ki, m, 6)
        sig, ki, m = valid_sig()
        add(NONCANON[rnd.randrange(len(NONCANON))] + sig[32:], ki, m, 7)
        sig, ki, m = valid_sig()
        add(SMALL_ORDER[rnd.randrange(len(SMALL_ORDER))] + sig[32:], ki, m, 8)
        m = rmsg()
        add(E.sign(key_seed(7), m), so_key, m, 9)
        m = rmsg()
        add(sign_mixed(ma, mbytes, mixed_j, m, rnd), mixed_key_idx, m, 10)
        sig, ki, m = valid_sig()
        add(sig, (ki + 1 + rnd.randrange(n_norm - 1)) % n_norm, m, 11)
        add(bytes(64), rnd.randrange(n_norm), rmsg(), 12)
        ki = rnd.randrange(n_norm); m = rmsg()
        add(sign_cofactored_only(secret_scalar(seeds[ki]), keys[ki], m, rnd), ki, m, 13)
        m = rmsg()
        add(sign_cofactored_only(ma, mbytes, m, rnd, mixed_j), mixed_key_idx, m, 14)
        sig, _, m = valid_sig()
        add(sig, nc_key, m, 15)
        sig, _, m = valid_sig()
        add(sig, noc_key, m, 16)
        sig, ki, m = valid_sig()
        sv = rnd.choice((0, E.L - 1))
        add(sig[:32] + sv.to_bytes(32, "little"), ki, m, 17)
        # s with bits 253..255 set: rejected by check_scalar; recoded naively its top comb digit would index
        # past the end of the base-point table
        sig, ki, m = valid_sig()
        s0 = int.from_bytes(sig[32:], "little")
        sv = rnd.choice((2**256 - 1, s0 + 2**253, s0 | 2**254, s0 | 2**255 | 2**254 | 2**253))
        add(sig[:32] + sv.to_bytes(32, "little"), ki, m, 19)

    # shuffle lanes so classes interleave within waves
    order = list(range(len(R)))
    rnd.shuffle(order)
    R = [R[i] for i in order]; S = [S[i] for i in order]; KI = [KI[i] for i in order]
    M = [M[i] for i in order]; CLS = [CLS[i] for i in order]
    exp = [1 if E.verify_strict(keys[KI[i]], R[i] + S[i], M[i]) else 0 for i in range(len(R))]
    key_ok = [1 if E.key_ok(k) else 0 for k in keys]
    stride = max(msg_len, 1)
    msg_arr = np.zeros((len(M), stride), dtype=np.uint8)
    for i, m in enumerate(M):
        msg_arr[i, :len(m)] = np.frombuffer(m, dtype=np.uint8) if m else 0
    return {
        "keys": np.frombuffer(b"".join(keys), dtype=np.uint8).reshape(-1, 32),
        "key_ok": np.array(key_ok, dtype=np.uint8),
        "R": np.frombuffer(b"".join(R), dtype=np.uint8).reshape(-1, 32),
        "S": np.frombuffer(b"".join(S), dtype=np.uint8).reshape(-1, 32),
        "key_idx": np.array(KI, dtype=np.uint16),
        "msg": msg_arr,
        "msg_len": np.array(msg_len, dtype=np.uint32),
        "expected": np.array(exp, dtype=np.uint8),
        "cls": np.array(CLS, dtype=np.uint8),
    }


def kats():
    out = {"rfc8032": [], "digest": {}, "rfc7693_blake2b512_abc": None}
    tests = [
        ("TEST 1", "9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60", ""),
        ("TEST 2", "4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb", "72"),
        ("TEST 3", "c5aa8df43f9f837bedb7442f31dcb7b166d38535076f094b85ce3a2e0b4458f7", "af82"),
    ]
    for name, sk, msg in tests:
        seed = bytes.fromhex(sk)
        out["rfc8032"].append({"name": name, "secret": sk, "public": E.public_key(seed).hex(),
                               "message": msg, "signature": E.sign(seed, bytes.fromhex(msg)).hex()})
    out["digest"] = {
        "operation": "testOperation",
        "blake2b512_hex": E.request_digest_hex(b"testOperation"),
        "sha256_hex": E.sha256(b"testOperation").hex(),
    }
    out["rfc7693_blake2b512_abc"] = E.request_digest(b"abc").hex()
    out["small_order_encodings"] = [b.hex() for b in SMALL_ORDER]
    out["noncanonical_decodable_encodings"] = [b.hex() for b in NONCANON]
    out["classes"] = {str(k): v for k, v in CLASSES.items()}
    return out


def main():
    rnd = random.Random(SEED)
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kats(), f, indent=1)
    batches = {}
    # msg_len 85 = the PBFT envelope (2 SHA-512 blocks); others exercise padding edges
    plan = [(85, 1024, 24), (0, 40, 2), (1, 40, 2), (47, 40, 2), (48, 40, 2), (111, 40, 2),
            (112, 40, 2), (175, 40, 2), (176, 40, 2), (300, 40, 2), (1023, 24, 1)]
    for ml, nv, na in plan:
        b = build_batch(rnd, ml, nv, na)
        for k, v in b.items():
            batches[f"m{ml}_{k}"] = v
        print(f"msg_len={ml}: {len(b['expected'])} sigs, {int(b['expected'].sum())} accept", flush=True)
    batches["msg_lens"] = np.array([p[0] for p in plan], dtype=np.uint32)
    np.savez_compressed(os.path.join(HERE, "verify_vectors.npz"), **batches)


if __name__ == "__main__":
    main()
