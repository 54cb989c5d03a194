#!/usr/bin/env python3
"""pbft_replica_push_many alone on the host (no GPU): config #4's 2^20 votes (n = 256, 2048 seqs x {Prepare,
Commit}, random signature bytes -- nothing is verified) pushed into one replica with a never-called verifier
override, the windows dropped between rounds by a stable checkpoint.  Prints ms per push_many.
usage: python tools/push_probe.py [rounds]"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import replica_sim
    L = replica_sim.lib()
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n, n_seq = 256, 2048
    rng = np.random.default_rng(1)
    keys = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    r = ctypes.c_void_p()
    assert L.pbft_replica_create(None, n, 0, keys.tobytes(), ctypes.byref(r)) == 0
    never = replica_sim.VERIFY_FN(lambda *a: -1)
    assert L.pbft_replica_set_verifier(r, never, None) == 0
    assert L.pbft_replica_set_log_window(r, 1 << 20) == 0
    N = 2 * n * n_seq
    sigs = rng.integers(0, 256, (N, 64), dtype=np.uint8)
    signer = np.tile(np.arange(n, dtype=np.uint32), 2 * n_seq)
    kind = np.tile(np.repeat(np.array([1, 2], np.uint8), n), n_seq)
    view = np.ones(N, np.uint64)
    times = []
    for rd in range(rounds + 1):
        seq = np.repeat(np.arange(1 + rd * n_seq, 1 + (rd + 1) * n_seq, dtype=np.uint64), 2 * n)
        dig = np.repeat(rng.integers(0, 256, (n_seq, 64), dtype=np.uint8), 2 * n, axis=0)
        q = ctypes.c_uint64()
        t = time.perf_counter()
        rc = L.pbft_replica_push_many(r, N, kind.ctypes.data, view.ctypes.data, seq.ctypes.data, dig.ctypes.data,
                                      signer.ctypes.data, sigs.ctypes.data, ctypes.byref(q))
        dt = (time.perf_counter() - t) * 1e3
        assert rc == 0 and q.value == N, (rc, q.value)
        if rd:
            times.append(dt)
        # drop the round's windows (stable checkpoint past them); the log window moves with it
        assert L.pbft_replica_stable_checkpoint(r, (rd + 1) * n_seq) == 0
    print(f"push_many 2^20 votes: median {np.median(times):.2f} ms, min {min(times):.2f}, "
          f"threads {os.environ.get('PBFT_REPLICA_THREADS', 'default')}")
    L.pbft_replica_destroy(r)


if __name__ == "__main__":
    main()
