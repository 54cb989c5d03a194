"""Config-#4 round with every adversarial class and special keys in the key set (TEST INFRASTRUCTURE).

Used by tests/test_gpu_verify.py::test_config4_every_lane_vs_oracle (VERDICT r04 "next round" item 1) and, at a
small size, by tests/test_oracle.py (the construction checked against both oracle restatements on the CPU).
The slots it certifies replace the reference's `validate_prepare` / `validate_commit`
(/root/reference/src/behavior.rs:159-195); the semantics are ed25519-dalek 1.0.1 `verify_strict`
(SURVEY.md Appendix A).

Special keys (SURVEY.md §8(d) adversarial classes "A small-order key" and "A mixed-order key with an
equation-valid signature"):
  * slot SMALL_SLOT: a small-order encoding -> key_ok 0, every signature under it rejects;
  * slot MIXED_SLOT: A' = aB + T (T of exact order 8) for the replica's own secret a.  The round's GPU signatures
    hash the old key bytes, so they reject under A'; `mixed_signatures` builds, in Python, equation-valid ones
    (R's torsion = -k T: cofactorless accept) and cofactored-only ones ([8](sB - kA' - R) = O but sB - kA' != R:
    reject).
"""
from __future__ import annotations

import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import ed25519_ref as E  # noqa: E402


def _torsion8():
    """A point of exact order 8: [L]Q for a curve point Q with a full torsion component."""
    y = 2
    while True:
        q = E.decompress(y.to_bytes(32, "little"))
        if q is not None:
            t = E.pt_mul(E.L, q)
            if not E.is_identity(E.pt_mul(4, t)):
                return t
        y += 1


T8 = _torsion8()
TORSION = [E.pt_mul(j, T8) for j in range(8)]
MIXED_J = 3  # A' = aB + [3]T8 (order 8)


def mixed_key(seed: bytes, j: int = MIXED_J):
    """(a, A' bytes) for A' = aB + [j]T8, a the RFC 8032 secret scalar of seed."""
    a = E.secret_expand(seed)[0]
    return a, E.compress(E.pt_add(E.pt_mul(a, E.BASE), TORSION[j]))


def mixed_signatures(a: int, A: bytes, msgs, valid: bool, seed: int, j: int = MIXED_J):
    """One signature per message under the mixed-order key A' = aB + [j]T8.

    valid: R = rB + T_i with i = -k j mod 8, so [s]B - [k]A' = rB - k[j]T8 = R exactly (cofactorless accept).
    not valid: R's torsion is any other i, so the equation holds only up to the torsion (cofactored-only: reject).
    """
    rnd = random.Random(seed)
    R, S = [], []
    for m in msgs:
        while True:
            r = rnd.randrange(1, E.L)
            rB = E.pt_mul(r, E.BASE)
            found = None
            for i in (range(8) if valid else rnd.sample(range(8), 8)):
                rb = E.compress(E.pt_add(rB, TORSION[i]))
                k = E.scalar_from_hash(E.sha512(rb + A + bytes(m)))
                if ((-(k * j)) % 8 == i) == valid:
                    found = (rb, (r + k * a) % E.L)
                    break
            if found:
                R.append(found[0])
                S.append(found[1].to_bytes(32, "little"))
                break
    return (np.frombuffer(b"".join(R), np.uint8).reshape(-1, 32).copy(),
            np.frombuffer(b"".join(S), np.uint8).reshape(-1, 32).copy())


def small_order_key() -> np.ndarray:
    """The identity point's encoding (y = 1): decodes, small order."""
    return np.frombuffer((1).to_bytes(32, "little"), np.uint8).copy()


def install_special_keys(seeds: np.ndarray, pub: np.ndarray, small_slot: int, mixed_slot: int):
    """pub with slot small_slot -> a small-order key and slot mixed_slot -> the mixed-order key of that replica's
    secret; returns (pub', a)."""
    pub2 = pub.copy()
    pub2[small_slot] = small_order_key()
    a, A = mixed_key(seeds[mixed_slot].tobytes())
    pub2[mixed_slot] = np.frombuffer(A, np.uint8)
    return pub2, a


def plant_mixed(R, S, key_idx, msg, msg_len, pub2, a, mixed_slot, n_valid, n_cofactored, seed):
    """Overwrite the first n_valid + n_cofactored lanes under mixed_slot (spread over the batch) with Python-built
    mixed-order signatures over those lanes' messages.  Returns (R', S', valid lanes, cofactored-only lanes)."""
    lanes = np.nonzero(key_idx == mixed_slot)[0]
    step = max(1, len(lanes) // (n_valid + n_cofactored))
    pick = lanes[::step][: n_valid + n_cofactored]
    v, c = pick[:n_valid], pick[n_valid:]
    A = pub2[mixed_slot].tobytes()
    R, S = R.copy(), S.copy()
    for lanes_k, valid, sd in ((v, True, seed), (c, False, seed + 1)):
        if len(lanes_k):
            r, s = mixed_signatures(a, A, [msg[i, :msg_len].tobytes() for i in lanes_k], valid, sd)
            R[lanes_k], S[lanes_k] = r, s
    return R, S, v, c
