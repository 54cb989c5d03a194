#!/usr/bin/env python3
"""Interleaved A/B of one pbft_verify_set_option on ONE context (same tables, same process), device-resident
launches of the config-#4 round's first n signatures (comb + finish per launch), per size.

usage: python tools/opt_ab.py OPTION VALUE_A VALUE_B [--sizes 131072,65536] [--rounds 8] [--iters 20]
e.g. tools/opt_ab.py 13 0 1   (PBFT_OPT_COMB_PRIO off / on)"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("option", type=int)
    ap.add_argument("a", type=int)
    ap.add_argument("b", type=int)
    ap.add_argument("--sizes", default="131072,65536,262144,1048576")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch
    import bench
    from pbft_amd import GpuBatchVerifier, bitmap_to_bool
    torch.cuda.set_device(0)
    seeds = bench.key_seeds(256)
    msg, key_idx = bench.envelopes(1, 2048, 256)
    v = GpuBatchVerifier(0)
    R, S, pub = v.sign(seeds, key_idx, msg, 85)
    assert v.set_keys(pub).all()
    dev = torch.device("cuda", 0)
    d = bench.to_device(torch, dev, R, S, key_idx, msg)
    st = torch.cuda.Stream(dev)
    for n in [int(x) for x in a.sizes.split(",")]:
        t = {a.a: [], a.b: []}
        bits = {}
        for r in range(a.rounds):
            for val in ((a.a, a.b) if r % 2 == 0 else (a.b, a.a)):
                v.set_option(a.option, val)
                ms, _ = bench.time_device(v, st, d, n, 3, torch)  # settle after the switch
                ms, _ = bench.time_device(v, st, d, n, a.iters, torch)
                t[val].append(ms)
                bits[val] = d["B"][: (n + 63) // 64].cpu().numpy().copy()
        assert (bits[a.a] == bits[a.b]).all() and bitmap_to_bool(bits[a.a].view(np.uint64), n).all(), n
        ma, mb = np.mean(t[a.a]), np.mean(t[a.b])
        print(f"n={n:8d} option {a.option}={a.a}: {ma:.4f} ms (min {min(t[a.a]):.4f})   ={a.b}: {mb:.4f} ms "
              f"(min {min(t[a.b]):.4f})   delta {100 * (mb - ma) / ma:+.1f} %", flush=True)
    v.close()


if __name__ == "__main__":
    main()
