#!/usr/bin/env python3
"""The 131k shard (one GPU of 8) launched back to back: interleaved A/B of the context's kernel-timing events
(PBFT_OPT_KERNEL_TIMING 1 vs 0: two event records per launch pair), then 200 launches for a rocprofv3 kernel trace
(tools/gap_stats.py reads the gaps between the comb's end, the finish's start and the next comb).
usage: python tools/shard_gap_probe.py [ab|trace|heat]   (heat: the shard timed as bench.py does -- first 131k
signatures of the 2^20 round, timing off -- cold, then after 3 s of back-to-back 2^20 rounds, then cold again)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from pbft_amd import GpuBatchVerifier
    mode = sys.argv[1] if len(sys.argv) > 1 else "ab"
    torch.cuda.set_device(0)
    n = 131072
    seeds = bench.key_seeds(256)
    msg, key_idx = bench.envelopes(1, 2048 if mode == "heat" else 256, 256)
    v = GpuBatchVerifier(0)
    R, S, pub = v.sign(seeds, key_idx, msg, 85)
    assert v.set_keys(pub).all()
    dev = torch.device("cuda", 0)
    d = bench.to_device(torch, dev, R, S, key_idx, msg)
    st = torch.cuda.Stream(dev)
    if mode == "trace":
        v.set_option(v.OPT_KERNEL_TIMING, 0)
        for _ in range(200):
            v.verify_device(d["R"].data_ptr(), d["S"].data_ptr(), d["K"].data_ptr(), d["M"].data_ptr(), 85, 85, n,
                            d["B"].data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        return
    if mode == "heat":
        v.set_option(v.OPT_KERNEL_TIMING, 0)
        def shard(tag):
            ks = [bench.time_device(v, st, d, n, 50, torch)[0] for _ in range(5)]
            print(f"{tag}: shard {np.median(ks):.4f} ms per launch pair (min {min(ks):.4f})", flush=True)
        shard("cold")
        t = time.perf_counter()
        while time.perf_counter() - t < 3.0:
            bench.time_device(v, st, d, len(msg), 10, torch)
        shard("after 3 s of 2^20 rounds")
        time.sleep(2.0)
        shard("after 2 s idle")
        return
    res = {0: [], 1: []}
    for rep in range(8):
        for t in ((1, 0) if rep % 2 == 0 else (0, 1)):
            v.set_option(v.OPT_KERNEL_TIMING, t)
            k, w = bench.time_device(v, st, d, n, 50, torch)
            res[t].append(k)
    for t in (1, 0):
        print(f"kernel timing {t}: {np.median(res[t]):.4f} ms per launch pair (min {min(res[t]):.4f})", flush=True)
    v.set_option(v.OPT_KERNEL_TIMING, 1)
    v.close()


if __name__ == "__main__":
    main()
