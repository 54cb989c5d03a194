#!/usr/bin/env python3
"""Rounds back to back, sequential vs pipelined (pbft_verify_batch_device_pipelined: comb on one stream, the finish
on a second one, so round k's finish can run under round k+1's comb), with finish configurations whose waves can
or cannot sit beside the comb's on a SIMD (VGPRs: finish<2,4,1> 263, finish<1,4,2> / <2,4,2> 206; the 131k comb
uses 2 waves x 128 of a SIMD's 512).  Interleaved, one context, wall time per round.
usage: python tools/pipe_shard_probe.py [sizes]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from pbft_amd import GpuBatchVerifier, bitmap_to_bool
    sizes = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [131072, 1 << 20]
    torch.cuda.set_device(0)
    seeds = bench.key_seeds(256)
    msg, key_idx = bench.envelopes(1, 2048, 256)
    v = GpuBatchVerifier(0)
    v.set_option(v.OPT_KERNEL_TIMING, 0)
    R, S, pub = v.sign(seeds, key_idx, msg, 85)
    assert v.set_keys(pub).all()
    dev = torch.device("cuda", 0)
    d = bench.to_device(torch, dev, R, S, key_idx, msg)
    st, fst = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    # (name, pipelined, finish width, finish waves per SIMD)
    cfgs = [("seq default", False, 0, 0), ("pipe default", True, 0, 0), ("pipe fm1 w2", True, 1, 2),
            ("pipe fm2 w2", True, 2, 2), ("seq fm1 w2", False, 1, 2), ("seq fm2 w2", False, 2, 2)]
    for n in sizes:
        res = {c[0]: [] for c in cfgs}
        for rep in range(4):
            for name, pipe, fm, w in (cfgs if rep % 2 == 0 else cfgs[::-1]):
                v.set_option(v.OPT_FINISH_WIDTH, fm)
                v.set_option(v.OPT_FINISH_WAVES, w)
                iters = 100 if n <= 262144 else 30
                for it in range(iters + 5):
                    if it == 5:
                        torch.cuda.synchronize()
                        t = time.perf_counter()
                    if pipe:
                        v.verify_device_pipelined(d["R"].data_ptr(), d["S"].data_ptr(), d["K"].data_ptr(),
                                                  d["M"].data_ptr(), 85, 85, n, d["B"].data_ptr(), st.cuda_stream,
                                                  fst.cuda_stream)
                    else:
                        v.verify_device(d["R"].data_ptr(), d["S"].data_ptr(), d["K"].data_ptr(), d["M"].data_ptr(),
                                        85, 85, n, d["B"].data_ptr(), st.cuda_stream)
                torch.cuda.synchronize()
                res[name].append((time.perf_counter() - t) * 1e3 / iters)
                assert bitmap_to_bool(d["B"][: (n + 63) // 64].cpu().numpy().view(np.uint64), n).all(), name
        base = np.mean(res["seq default"])
        for name, x in res.items():
            print(f"n={n:8d} {name:14s} {np.mean(x):.4f} ms/round (min {min(x):.4f})  {100 * (np.mean(x) - base) / base:+.1f} %",
                  flush=True)
    v.set_option(v.OPT_FINISH_WIDTH, 0)
    v.set_option(v.OPT_FINISH_WAVES, 0)
    v.close()


if __name__ == "__main__":
    main()
