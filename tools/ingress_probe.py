#!/usr/bin/env python3
"""GPU probe: bench.py's replica legs alone (replica_ingress_2^20: one message per call on one thread; and the
push_many replica_flush_2^20 leg with its max-round phases), printed as one JSON line.  Usage:
python tools/ingress_probe.py [--seqs 2048] [--skip-flush-leg]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seqs", type=int, default=bench.SEQS)
    ap.add_argument("--skip-flush-leg", action="store_true")
    ap.add_argument("--modes", default="")
    ap.add_argument("--skip-ingress-leg", action="store_true")
    ap.add_argument("--flush-ab", default="", help="ENV=v1,v2,...: the flush leg cycled over these values")
    ap.add_argument("--rounds", type=int, default=9)
    a = ap.parse_args()
    import torch  # noqa: F401
    from pbft_amd import GpuBatchVerifier
    n_rep = bench.N_REPLICAS
    seeds = bench.key_seeds(n_rep)
    msg, key_idx = bench.envelopes(1, a.seqs, n_rep)
    v = GpuBatchVerifier(0)
    v.set_option(v.OPT_KERNEL_TIMING, 0)
    R, S_good, pub = v.sign(seeds, key_idx, msg, bench.ENVELOPE)
    S, bad = bench.corrupt(S_good, bench.ADV_FRAC, bench.SEED)
    expect = np.ones(len(msg), bool)
    expect[bad] = False
    assert v.set_keys(pub).all()
    out = {}
    if not a.skip_flush_leg:
        fa = {}
        if a.flush_ab:
            env, vals = a.flush_ab.split("=")
            fa = {"modes": vals.split(","), "mode_env": env}
        out["replica_flush_2^20"] = bench.replica_round_leg(v, seeds, pub, R, S, key_idx, msg, expect,
                                                            rounds=a.rounds, **fa)
        if a.skip_ingress_leg:
            print(json.dumps(out), flush=True)
            v.close()
            return
    modes = None
    if a.modes:
        modes = [("push", 2, True)] + [(m, 2, False) for m in a.modes.split(",")]
    out["replica_ingress_2^20"] = bench.replica_ingress_leg(v, seeds, pub, S, ~expect, a.seqs, modes)
    print(json.dumps(out), flush=True)
    v.close()


if __name__ == "__main__":
    main()
