#!/usr/bin/env python3
"""The bench's replica leg (bench.replica_round_leg: config #4's 2^20-vote round through ONE pbft_replica) alone,
with the replica's flush timeline on stderr (PBFT_REPLICA_TRACE=1: submit, fill / launch per 2^18-row step, each
landed chunk applied, finish, evaluate, gc -- ms from the submit).   usage: python tools/replica_probe.py [rounds]"""
import json
import os
import sys

os.environ.setdefault("PBFT_REPLICA_TRACE", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    from pbft_amd import GpuBatchVerifier
    torch.cuda.set_device(0)
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    n_ctx = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    modes, mode_env = None, "PBFT_REPLICA_DIRECT"
    if len(sys.argv) > 3:
        spec = sys.argv[3]
        if "=" in spec:
            mode_env, spec = spec.split("=", 1)
        modes = spec.split(",")
    seeds = bench.key_seeds(bench.N_REPLICAS)
    msg, key_idx = bench.envelopes(1, bench.SEQS, bench.N_REPLICAS)
    v = GpuBatchVerifier(0)
    R, S_good, pub = v.sign(seeds, key_idx, msg, bench.ENVELOPE)
    S, bad = bench.corrupt(S_good, bench.ADV_FRAC, bench.SEED)
    expect = np.ones(len(msg), bool)
    expect[bad] = False
    assert v.set_keys(pub).all()
    print(json.dumps(bench.replica_round_leg(v, seeds, pub, R, S, key_idx, msg, expect, rounds=rounds,
                                               n_ctx=n_ctx, modes=modes, mode_env=mode_env)), flush=True)
    v.close()


if __name__ == "__main__":
    main()
