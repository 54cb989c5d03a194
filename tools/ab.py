#!/usr/bin/env python3
"""Interleaved A/B timing of verify_kernel builds in ONE process (cdna guide §5.4 rule 24).

usage: python tools/ab.py lib1.so lib2.so[@opt=value,...] ... [--rounds 8 --iters 10 --budget-mb X]
Each lib gets its own context (and its own 30-GB base-point table: with several libs give each a key-table
budget, e.g. @3=20000 = the 16-position plan, or the second lib cannot allocate) on the same synthetic 2^20-signature round; `@2=4,4=6,8=2` sets
pbft_verify_set_option(option, value) pairs on that context (the same library may appear with different options).
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--replicas", type=int, default=256)
    ap.add_argument("--seqs", type=int, default=2048)
    ap.add_argument("--per-launch-events", action="store_true", help="also record a torch event pair per launch")
    ap.add_argument("--sizes", default="", help="comma list of batch sizes (default: the whole round)")
    ap.add_argument("--votes", action="store_true", help="time the votes form (pbft_verify_votes_device)")
    ap.add_argument("--latency", action="store_true", help="p50 wall time of single synchronized launches")
    a = ap.parse_args()
    import torch
    import bench
    from pbft_amd import GpuBatchVerifier, bitmap_to_bool
    torch.cuda.set_device(0)
    seeds = bench.key_seeds(a.replicas)
    msg, key_idx = bench.envelopes(1, a.seqs, a.replicas)
    n = len(msg)
    v0 = GpuBatchVerifier(0)
    R, S, pub = v0.sign(seeds, key_idx, msg, 85)
    v0.close()
    dev = torch.device("cuda", 0)
    dR, dS = torch.from_numpy(R).to(dev), torch.from_numpy(S).to(dev)
    dK = torch.from_numpy(key_idx.view(np.int16)).to(dev)
    mp = np.zeros(n * 85 + 64, dtype=np.uint8)
    mp[: n * 85] = msg.reshape(-1)
    dM = torch.from_numpy(mp).to(dev)
    dB = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
    env, inv = np.unique(msg, axis=0, return_inverse=True)
    ep = np.zeros(len(env) * 85 + 64, dtype=np.uint8)
    ep[: len(env) * 85] = env.reshape(-1)
    dE = torch.from_numpy(ep).to(dev)
    dI = torch.from_numpy(inv.reshape(-1).astype(np.int32)).to(dev)
    torch.cuda.synchronize()
    st = torch.cuda.Stream(dev)
    ctxs = []
    for p in a.libs:
        path, _, opts = p.partition("@")
        lib = ctypes.CDLL(os.path.abspath(path))
        vp = ctypes.c_void_p
        lib.pbft_verify_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
        lib.pbft_verify_set_keys.argtypes = [vp, vp, ctypes.c_uint32, vp]
        lib.pbft_verify_batch_device.argtypes = [vp, vp, vp, vp, vp, ctypes.c_uint32, ctypes.c_uint32,
                                                 ctypes.c_uint64, vp, vp]
        lib.pbft_verify_votes_device.argtypes = [vp, vp, vp, vp, vp, vp, ctypes.c_uint32, ctypes.c_uint64, vp, vp]
        lib.pbft_build_info.restype = ctypes.c_char_p
        c = vp()
        assert lib.pbft_verify_ctx_create(0, ctypes.byref(c)) == 0
        lib.pbft_verify_set_option.argtypes = [vp, ctypes.c_int, ctypes.c_uint64]
        for kv in filter(None, opts.split(",")):
            k, v = kv.split("=")
            assert lib.pbft_verify_set_option(c, int(k), int(v)) == 0, kv
        ok = np.zeros(len(pub), np.uint8)
        assert lib.pbft_verify_set_keys(c, pub.ctypes.data, len(pub), ok.ctypes.data) == 0
        ctxs.append((p, lib, c))
    sizes = [int(x) for x in a.sizes.split(",")] if a.sizes else [n]
    full = n
    if a.latency:
        import time
        for n in sizes:
            lat = {p: [] for p in a.libs}
            for r in range(a.rounds * 25):
                for p, lib, c in ctxs:
                    torch.cuda.synchronize()
                    t = time.perf_counter()
                    assert lib.pbft_verify_batch_device(c, dR.data_ptr(), dS.data_ptr(), dK.data_ptr(), dM.data_ptr(),
                                                        85, 85, n, dB.data_ptr(), st.cuda_stream) == 0
                    st.synchronize()
                    lat[p].append((time.perf_counter() - t) * 1e3)
            for p, lib, c in ctxs:
                t = np.array(lat[p][10:])
                print(f"N={n:8d} {os.path.basename(p):32s} p50 {np.median(t):.4f} ms  p99 {np.percentile(t, 99):.4f}",
                      flush=True)
        return
    for n in sizes:
      res = {p: [] for p in a.libs}
      for r in range(a.rounds):
        for p, lib, c in ctxs:
            dB.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.iters):
                if a.per_launch_events:
                    torch.cuda.Event(enable_timing=True).record(st)
                if a.votes:
                    assert lib.pbft_verify_votes_device(c, dR.data_ptr(), dS.data_ptr(), dK.data_ptr(), dI.data_ptr(),
                                                        dE.data_ptr(), len(env), n, dB.data_ptr(), st.cuda_stream) == 0
                else:
                    assert lib.pbft_verify_batch_device(c, dR.data_ptr(), dS.data_ptr(), dK.data_ptr(), dM.data_ptr(),
                                                        85, 85, n, dB.data_ptr(), st.cuda_stream) == 0
            e1.record(st)
            st.synchronize()
            res[p].append(e0.elapsed_time(e1) / a.iters)
            if "abl" not in os.path.basename(p):
                assert bitmap_to_bool(dB.cpu().numpy().view(np.uint64), n).all(), p
      for p, lib, c in ctxs:
        t = np.array(res[p])
        print(f"N={n:8d} {os.path.basename(p):32s} median {np.median(t):.4f} ms  min {t.min():.4f}  "
              f"-> {n / np.median(t) * 1e3 / 1e6:.1f} M verifies/s   [{lib.pbft_build_info().decode()}]", flush=True)
        if hasattr(lib, "pbft_debug_fin_stamps"):
            # finish-kernel phase stamps of the last launch (PBFT_FIN_STAMPS build): per wave, shader cycles
            waves = 4096
            buf = np.zeros((waves, 12), np.uint64)
            lib.pbft_debug_fin_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_uint32(waves))
            live = buf[(buf[:, 5] > buf[:, 0]) & (buf[:, 0] > 0)]
            if len(live):
                d = np.diff(live[:, :6].astype(np.int64), axis=1)
                names = ["prefix", "tree-up", "inversion", "tree-down", "back+compare"]
                med = ", ".join(f"{nm} {int(np.median(d[:, k]))}" for k, nm in enumerate(names))
                span = (live[:, 7].max() - live[:, 6].min()) / 100.0  # s_memrealtime: 100 MHz
                first = (live[:, 6].max() - live[:, 6].min()) / 100.0
                print(f"    finish stamps ({len(live)} waves, median shader cycles): {med}; "
                      f"total {int(np.median(live[:, 5].astype(np.int64) - live[:, 0].astype(np.int64)))}; "
                      f"wall span {span:.1f} us, wave starts spread {first:.1f} us; inversion: divsteps "
                      f"{int(np.median(live[:, 8]))}, updates {int(np.median(live[:, 9]))} cycles over "
                      f"{int(np.median(live[:, 10]))} batches", flush=True)


if __name__ == "__main__":
    main()
