#!/usr/bin/env python3
"""Throughput of back-to-back 2^20-signature rounds on 1 stream vs 2 streams (two cloned contexts, alternating
rounds, so one round's finish_kernel can overlap the next round's comb_kernel)."""
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
    torch.cuda.set_device(0)
    seeds = bench.key_seeds(256)
    msg, key_idx = bench.envelopes(1, 2048, 256)
    n = len(msg)
    v = GpuBatchVerifier(0)
    R, S, pub = v.sign(seeds, key_idx, msg, 85)
    v.set_keys(pub)
    c2 = v.clone()
    dev = torch.device("cuda", 0)
    dR, dS = torch.from_numpy(R).to(dev), torch.from_numpy(S).to(dev)
    dK = torch.from_numpy(key_idx.view(np.int16)).to(dev)
    mp = np.zeros(n * 85 + 64, np.uint8)
    mp[: n * 85] = msg.reshape(-1)
    dM = torch.from_numpy(mp).to(dev)
    dB = [torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev) for _ in range(2)]
    st = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    ctx = [v, c2]

    def run(k, two):
        j = k % 2 if two else 0
        ctx[j].verify_device(dR.data_ptr(), dS.data_ptr(), dK.data_ptr(), dM.data_ptr(), 85, 85, n, dB[j].data_ptr(),
                             st[j].cuda_stream)

    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        run(0, False)
        torch.cuda.synchronize()
    for two in (False, True, False, True):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(40):
            run(k, two)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 40
        assert bitmap_to_bool(dB[0].cpu().numpy().view(np.uint64), n).all()
        print(f"{'2 streams' if two else '1 stream '}: {dt * 1e3:.4f} ms/round  {n / dt / 1e6:.1f} M verifies/s")


if __name__ == "__main__":
    main()
