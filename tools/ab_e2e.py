#!/usr/bin/env python3
"""PCIe-inclusive 2^20 round (bench.py e2e_host_round / e2e_votes_round) for the library in PBFT_VERIFY_LIB: one
library per process (the key tables of one context fill the HBM); prints one line per leg."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    from pbft_amd import GpuBatchVerifier
    torch.cuda.set_device(0)
    seeds = bench.key_seeds(256)
    msg, key_idx = bench.envelopes(1, 2048, 256)
    v = GpuBatchVerifier(0)
    R, S, pub = v.sign(seeds, key_idx, msg, 85)
    assert v.set_keys(pub).all()
    expect = np.ones(len(R), bool)
    lib = os.path.basename(os.environ.get("PBFT_VERIFY_LIB", "libpbft_verify.so"))
    for name, fn in (("e2e_soa", bench.e2e_host_round), ("e2e_votes", bench.e2e_votes_round)):
        r = fn(v, R, S, key_idx, msg, expect, torch, iters=9)
        print(f"{lib:24s} {name:10s} {r['ms_per_round']:.3f} ms  {r['value'] / 1e6:.1f} M/s", flush=True)
    v.close()


if __name__ == "__main__":
    main()
