#!/usr/bin/env python3
"""Verify-launch time vs batch size and finish width (device-resident, 2^20-signature config-#4 round).

usage: python tools/size_probe.py [--iters 20]   (run under rocprofv3 --kernel-trace to split comb / finish)
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--sizes", default="32768,65536,131072,262144,524288,1048576")
    ap.add_argument("--widths", default="1,4,16")
    ap.add_argument("--trees", default="0", help="finish cross-lane tree levels to sweep (PBFT_OPT_FINISH_TREE)")
    ap.add_argument("--split-below", type=int, default=-1, help="PBFT_OPT_SPLIT_BELOW for this run (-1: default)")
    a = ap.parse_args()
    import torch
    import bench
    from pbft_amd import GpuBatchVerifier, bitmap_to_bool
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    seeds = bench.key_seeds(256)
    msg, key_idx = bench.envelopes(1, 2048, 256)
    v = GpuBatchVerifier(0)
    R, S, pub = v.sign(seeds, key_idx, msg, 85)
    assert v.set_keys(pub).all()
    d = bench.to_device(torch, dev, R, S, key_idx, msg)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    if a.split_below >= 0:
        v.set_option(v.OPT_SPLIT_BELOW, a.split_below)
    bench.time_device(v, st, d, len(R), 20, torch)  # settle
    out = []
    for n in [int(x) for x in a.sizes.split(",")]:
        for fm, lv in [(int(x), int(y)) for y in a.trees.split(",") for x in a.widths.split(",")]:
            v.set_option(v.OPT_FINISH_WIDTH, fm)
            v.set_option(v.OPT_FINISH_TREE, lv)
            bench.time_device(v, st, d, n, 3, torch)
            ms, wall = bench.time_device(v, st, d, n, a.iters, torch)
            ok = bitmap_to_bool(d["B"].cpu().numpy().view(np.uint64), n).all()
            out.append({"n": n, "fin_m": fm, "fin_tree": lv, "split_below": a.split_below, "ms": ms, "wall_ms": wall, "verifies_per_s": n / (ms * 1e-3), "ok": bool(ok)})
            print(json.dumps(out[-1]), flush=True)
    v.set_option(v.OPT_FINISH_WIDTH, 0)
    v.set_option(v.OPT_FINISH_TREE, 7)
    v.close()


if __name__ == "__main__":
    main()
