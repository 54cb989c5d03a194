#!/usr/bin/env python3
"""p50/p99 of a 4096-signature device-resident round: direct launches vs one HIP-graph replay."""
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
    n_rep, n_seq = 256, 8
    seeds = bench.key_seeds(n_rep)
    msg, key_idx = bench.envelopes(1, n_seq, n_rep)
    n = len(msg)  # 4096
    v = GpuBatchVerifier(0)
    R, S, pub = v.sign(seeds, key_idx, msg, 85)
    v.set_keys(pub)
    dev = torch.device("cuda", 0)
    dR, dS = torch.from_numpy(R).to(dev), torch.from_numpy(S).to(dev)
    dK = torch.from_numpy(key_idx.view(np.int16)).to(dev)
    mp = np.zeros(n * 85 + 64, np.uint8)
    mp[: n * 85] = msg.reshape(-1)
    dM = torch.from_numpy(mp).to(dev)
    dB = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
    st = torch.cuda.Stream(dev)
    v.reserve(n)

    def launch(stream):
        v.verify_device(dR.data_ptr(), dS.data_ptr(), dK.data_ptr(), dM.data_ptr(), 85, 85, n, dB.data_ptr(),
                        stream)

    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        launch(torch.cuda.current_stream().cuda_stream)
    for mode in ("direct", "graph", "direct", "graph"):
        lat = []
        for it in range(400):
            torch.cuda.synchronize()
            t = time.perf_counter()
            if mode == "graph":
                g.replay()
            else:
                launch(st.cuda_stream)
            torch.cuda.synchronize()
            lat.append((time.perf_counter() - t) * 1e3)
        lat = np.array(lat[20:])
        assert bitmap_to_bool(dB.cpu().numpy().view(np.uint64), n).all()
        print(f"{mode:7s} p50 {np.median(lat):.4f} ms  p99 {np.percentile(lat, 99):.4f} ms")


if __name__ == "__main__":
    main()
