#!/usr/bin/env python3
"""Config #5 legs alone (bench.stream_latency: back-to-back and 2^21/s offered, 4096-signature host batches over 4
contexts), N one-second samples: the latency distribution under the current PBFT_SPIN_WAIT (run once per mode, in
alternating processes).   usage: python tools/stream_ab.py [samples]"""
import json
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    seeds = bench.key_seeds(256)
    msg, key_idx = bench.envelopes(1, 2048, 256)
    v = GpuBatchVerifier(0)
    v.set_option(v.OPT_KERNEL_TIMING, 0)
    R, S, pub = v.sign(seeds, key_idx, msg, 85)
    assert v.set_keys(pub).all()
    out = {"spin": os.environ.get("PBFT_SPIN_WAIT", "1")}
    for name, rate in (("back_to_back", float("inf")), ("offered_2^21", 2.0 ** 21)):
        xs = [bench.stream_latency(v, R, S, key_idx, msg, rate) for _ in range(reps)]
        out[name] = {k: [round(x[k], 4) for x in xs] for k in ("p50_ms", "p99_ms", "p999_ms", "max_ms")}
    print(json.dumps(out), flush=True)
    v.close()


if __name__ == "__main__":
    main()
