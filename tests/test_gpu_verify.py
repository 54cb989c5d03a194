"""GPU parity: the HIP verifier's bitmap vs the oracle, bit-exact.

Oracle = oracle/ed25519_ref.py (expected bits committed in tests/golden) and
oracle/ed25519_oracle.c for seeded batches too large for pure Python.
"""
import ctypes
import hashlib
import os

import numpy as np
import pytest

from conftest import ROOT, golden_batches

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gv():
    from pbft_amd import GpuBatchVerifier
    v = GpuBatchVerifier(0)
    yield v
    v.close()


def test_golden_bitmaps_bit_exact(gv, golden):
    from pbft_amd import SigBatch, bitmap_to_bool
    for ml, b in golden_batches(golden):
        ok = gv.set_keys(b["keys"])
        assert (ok == b["key_ok"].astype(bool)).all(), ml
        bm = gv.verify(SigBatch(b["R"], b["S"], b["key_idx"], b["msg"], ml))
        got = bitmap_to_bool(bm, len(b["R"]))
        exp = b["expected"].astype(bool)
        bad = np.nonzero(got != exp)[0]
        assert len(bad) == 0, (ml, bad[:10], b["cls"][bad[:10]])
        # bits past N are zero
        n = len(b["R"])
        if n % 64:
            assert int(bm[-1]) >> (n % 64) == 0
