#!/usr/bin/env python3
"""Config #5 leg alone (bench.py stream_latency): 4096-signature host-buffer batches at 2^21 signatures/s over 4
cloned contexts, pinned inputs, repeated; prints p50 / p99 / p99.9 / max per repetition."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from pbft_amd import GpuBatchVerifier
    torch.cuda.set_device(0)
    seeds = bench.key_seeds(256)
    msg, key_idx = bench.envelopes(1, 2048, 256)
    v = GpuBatchVerifier(0)
    R, S, pub = v.sign(seeds, key_idx, msg, 85)
    budget = int(os.environ.get("PBFT_KEY_TABLE_BUDGET_MB", "0"))
    if budget:
        v.set_option(v.OPT_KEY_TABLE_BUDGET_MB, budget)
    assert v.set_keys(pub).all()
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dur = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
    for r in range(reps):
        s = bench.stream_latency(v, R, S, key_idx, msg, float(1 << 21), duration_s=dur)
        print(f"rep {r}: batches {s['batches']} p50 {s['p50_ms']:.4f} p99 {s['p99_ms']:.4f} p99.9 {s['p999_ms']:.4f} "
              f"max {s['max_ms']:.4f} ms (p99/p50 {s['p99_ms'] / s['p50_ms']:.2f})", flush=True)
    v.close()


if __name__ == "__main__":
    main()
