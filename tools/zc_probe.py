#!/usr/bin/env python3
"""Zero-copy votes rows (PBFT_OPT_VOTES_ZERO_COPY) against chunked H2D, interleaved in one process: config #4's
2^20-vote round staged in the context's pinned staging (pbft_verify_votes_stage), then submit + wait timed
(the GPU pipeline alone: the fill is done before the clock starts), and the pageable pbft_verify_votes call
(copy into the staging + the same pipeline).  Every bitmap is checked against the corrupted positions.
usage: python tools/zc_probe.py [rounds] [settings, default 1,0]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    from pbft_amd import GpuBatchVerifier, bitmap_to_bool
    torch.cuda.set_device(0)
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    settings = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,0").split(",")]
    seeds = bench.key_seeds(bench.N_REPLICAS)
    msg, key_idx = bench.envelopes(1, bench.SEQS, bench.N_REPLICAS)
    v = GpuBatchVerifier(0)
    R, S_good, pub = v.sign(seeds, key_idx, msg, bench.ENVELOPE)
    S, bad = bench.corrupt(S_good, bench.ADV_FRAC, bench.SEED)
    expect = np.ones(len(msg), bool)
    expect[bad] = False
    assert v.set_keys(pub).all()
    env, inv = np.unique(msg, axis=0, return_inverse=True)
    inv = inv.reshape(-1).astype(np.uint32)
    n, ne = len(msg), len(env)
    res = {zc: {"staged": [], "pageable": []} for zc in settings}
    for r in range(rounds + 1):
        for zc in settings:
            v.set_option(v.OPT_VOTES_ZERO_COPY, zc)
            st = v.stage_votes(n, ne)
            st["sig"][:, :32] = R
            st["sig"][:, 32:] = S
            st["key_idx"][:] = key_idx
            st["env_idx"][:] = inv
            st["envelopes"][:] = env
            t = time.perf_counter()
            out = v.wait(v.submit_staged(n, ne))
            dt = (time.perf_counter() - t) * 1e3
            assert (bitmap_to_bool(out, n) == expect).all(), ("staged", zc)
            t = time.perf_counter()
            out = v.verify_votes(R, S, key_idx, inv, env)
            dp = (time.perf_counter() - t) * 1e3
            assert (bitmap_to_bool(out, n) == expect).all(), ("pageable", zc)
            if r:
                res[zc]["staged"].append(dt)
                res[zc]["pageable"].append(dp)
    out = {}
    for zc in settings:
        for k, x in res[zc].items():
            x = np.array(x)
            out[f"zc{zc}_{k}_ms"] = {"median": float(np.median(x)), "min": float(x.min()), "max": float(x.max()),
                                     "verifies_per_s": n / float(np.median(x)) * 1e3}
    print(json.dumps(out, indent=1), flush=True)
    v.close()


if __name__ == "__main__":
    main()
