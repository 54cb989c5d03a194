#!/usr/bin/env python3
"""Launch gaps: K back-to-back pbft_verify_batch_device launches (comb + finish) timed by one HIP event pair,
against the same launches captured into a HIP graph (torch.cuda.CUDAGraph) and replayed, at the 131k shard and the
2^20 round (config #4 rows, 13-position plan).  Prints ms per launch for both and checks every bitmap.
usage: python tools/graph_probe.py [K]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    from pbft_amd import GpuBatchVerifier, bitmap_to_bool
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    seeds = bench.key_seeds(bench.N_REPLICAS)
    msg, key_idx = bench.envelopes(1, bench.SEQS, bench.N_REPLICAS)
    v = GpuBatchVerifier(0)
    v.set_option(v.OPT_KERNEL_TIMING, 0)
    R, S_good, pub = v.sign(seeds, key_idx, msg, bench.ENVELOPE)
    S, bad = bench.corrupt(S_good, bench.ADV_FRAC, bench.SEED)
    expect = np.ones(len(msg), bool)
    expect[bad] = False
    assert v.set_keys(pub).all()
    d = bench.to_device(torch, dev, R, S, key_idx, msg)
    st = torch.cuda.Stream(dev)
    out = {}
    for n in (131072, len(msg)):
        v.reserve(n)

        def launch():
            v.verify_device(d["R"].data_ptr(), d["S"].data_ptr(), d["K"].data_ptr(), d["M"].data_ptr(),
                            bench.ENVELOPE, bench.ENVELOPE, n, d["B"].data_ptr(), st.cuda_stream)
        with torch.cuda.stream(st):
            for _ in range(3):
                launch()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for _ in range(K):
                launch()
        torch.cuda.synchronize()
        res = {"eager": [], "graph": []}
        for rep in range(6):
            for mode in ("eager", "graph"):
                d["B"].zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record(st)
                if mode == "graph":
                    with torch.cuda.stream(st):
                        g.replay()
                else:
                    for _ in range(K):
                        launch()
                e1.record(st)
                torch.cuda.synchronize()
                got = bitmap_to_bool(d["B"].cpu().numpy().view(np.uint64), n)
                assert (got == expect[:n]).all(), (mode, n)
                if rep:
                    res[mode].append(e0.elapsed_time(e1) / K)
        out[str(n)] = {m: float(np.median(x)) for m, x in res.items()}
        del g
    print(json.dumps(out, indent=1), flush=True)
    v.close()


if __name__ == "__main__":
    main()
