#!/usr/bin/env python3
"""r06 probe: why bench.py's replica_flush_2^20 leg runs slower inside the bench process than in a fresh one.
Runs the leg, then ~N seconds of the headline's device-resident 2^20 launches (the GPU's heavy phase before the leg
in bench.py), then the leg again, and prints the two legs' medians / means / phases as one JSON line.
usage: python tools/replica_heat_probe.py [--heat-s 8] [--rounds 20]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def summary(r):
    return {"ms_per_round": r["ms_per_round"], "ms_per_round_mean": r["ms_per_round_mean"],
            "min_max": r["ms_per_round_min_max"], "push_many_ms": r["push_many_ms"], "flush_ms": r["flush_ms"],
            "max_round": r["max_round"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--heat-s", type=float, default=8.0)
    ap.add_argument("--rounds", type=int, default=20)
    a = ap.parse_args()
    import torch
    from pbft_amd import GpuBatchVerifier
    n_rep = bench.N_REPLICAS
    seeds = bench.key_seeds(n_rep)
    msg, key_idx = bench.envelopes(1, bench.SEQS, n_rep)
    v = GpuBatchVerifier(0)
    R, S_good, pub = v.sign(seeds, key_idx, msg, bench.ENVELOPE)
    S, bad = bench.corrupt(S_good, bench.ADV_FRAC, bench.SEED)
    expect = np.ones(len(msg), bool)
    expect[bad] = False
    assert v.set_keys(pub).all()
    out = {"fresh": summary(bench.replica_round_leg(v, seeds, pub, R, S, key_idx, msg, expect, rounds=a.rounds))}
    dev = torch.device("cuda", 0)
    d = bench.to_device(torch, dev, R, S, key_idx, msg)
    stream = torch.cuda.Stream(dev)
    t = time.perf_counter()
    launches = 0
    while time.perf_counter() - t < a.heat_s:
        bench.time_device(v, stream, d, len(R), 50, torch)
        launches += 50
    out["heat"] = {"seconds": time.perf_counter() - t, "launches": launches}
    out["after_heat"] = summary(bench.replica_round_leg(v, seeds, pub, R, S, key_idx, msg, expect, rounds=a.rounds))
    time.sleep(3.0)
    out["after_rest"] = summary(bench.replica_round_leg(v, seeds, pub, R, S, key_idx, msg, expect, rounds=a.rounds))
    print(json.dumps(out), flush=True)
    v.close()


if __name__ == "__main__":
    main()
