#!/usr/bin/env python3
"""Config #5 back-to-back leg (bench.py stream_latency with offered rate = inf) with every host call timed: where do
the 7.5-9.4 ms maxima of `stream_4k.back_to_back.max_ms` come from?

Run with PBFT_LAUNCH_TRACE=<us> to have the library report each of its HIP calls slower than that on stderr.
usage: tools/stall_probe.py [reps] [seconds] [pinned 1|0]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def leg(v, batches, dur, n_ctx=4):
    import numpy as np
    ctxs = [v.clone() for _ in range(n_ctx)]
    for c in ctxs:
        c.wait(c.submit(batches[0]))
    pending = [None] * n_ctx
    calls = []   # (duration ms, what, t since start ms)
    lat = []
    import gc
    gc.collect()
    gc.disable()
    t0 = time.perf_counter()
    k = 0
    while True:
        now = time.perf_counter()
        for ci, p in enumerate(pending):
            if p is not None:
                a = time.perf_counter()
                out = ctxs[ci].poll(p[0])
                b = time.perf_counter()
                calls.append(((b - a) * 1e3, f"poll ctx{ci}", (a - t0) * 1e3))
                if out is not None:
                    lat.append(((b - p[1]) * 1e3, (p[1] - t0) * 1e3, ci))
                    pending[ci] = None
        if now - t0 >= dur:
            if all(p is None for p in pending):
                break
            continue
        ci = k % n_ctx
        if pending[ci] is not None:
            a = time.perf_counter()
            ctxs[ci].wait(pending[ci][0])
            b = time.perf_counter()
            calls.append(((b - a) * 1e3, f"wait ctx{ci}", (a - t0) * 1e3))
            lat.append(((b - pending[ci][1]) * 1e3, (pending[ci][1] - t0) * 1e3, ci))
        a = time.perf_counter()
        t = ctxs[ci].submit(batches[k % len(batches)])
        b = time.perf_counter()
        calls.append(((b - a) * 1e3, f"submit ctx{ci}", (a - t0) * 1e3))
        pending[ci] = (t, a)
        k += 1
    gc.enable()
    for c in ctxs:
        c.close()
    la = np.array([x[0] for x in lat])
    print(f"  batches {len(lat)} p50 {np.median(la):.4f} p99 {np.percentile(la, 99):.4f} "
          f"p99.9 {np.percentile(la, 99.9):.4f} max {la.max():.4f} ms", flush=True)
    for d, ts, ci in sorted(lat, reverse=True)[:4]:
        print(f"  slow batch: {d:.3f} ms, submitted at {ts:.1f} ms on ctx{ci}", flush=True)
    calls.sort(reverse=True)
    for d, what, ts in calls[:8]:
        print(f"  slow call: {what} {d:.3f} ms at {ts:.1f} ms", flush=True)
    # gaps in the loop itself (the thread not running for a while)
    return la.max()


def main():
    import numpy as np
    import torch
    import bench
    from pbft_amd import GpuBatchVerifier, SigBatch
    torch.cuda.set_device(0)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dur = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    pinned = (sys.argv[3] if len(sys.argv) > 3 else "1") == "1"
    seeds = bench.key_seeds(256)
    msg, key_idx = bench.envelopes(1, 2048, 256)
    v = GpuBatchVerifier(0)
    R, S, pub = v.sign(seeds, key_idx, msg, 85)
    assert v.set_keys(pub).all()
    m = 64 * 4096
    R, S, key_idx, msg = R[:m], S[:m], key_idx[:m], msg[:m]
    if pinned:
        pin = lambda a: torch.from_numpy(np.ascontiguousarray(a)).pin_memory().numpy()  # noqa: E731
        R, S, key_idx, msg = pin(R), pin(S), pin(key_idx), pin(msg)
    batches = [SigBatch(R[i * 4096:(i + 1) * 4096], S[i * 4096:(i + 1) * 4096], key_idx[i * 4096:(i + 1) * 4096],
                        msg[i * 4096:(i + 1) * 4096], 85) for i in range(64)]
    for r in range(reps):
        print(f"rep {r} ({'pinned' if pinned else 'pageable'}, {dur} s back to back):", flush=True)
        leg(v, batches, dur)
    v.close()


if __name__ == "__main__":
    main()
