#!/usr/bin/env python3
"""Phase stamps of comb_kernel waves (diagnostic build: tools/build_variant.sh stamps -DPBFT_COMB_STAMPS=1) at the
131k shard and at 2^20 (attribute the shard's stalls before trying another kernel shape).

Per size: the in-kernel clock (delta s_memtime / delta s_memrealtime x 100 MHz, median over waves), and per wave the
shader cycles of its phases -- hash + recoding, gather waits (vmcnt(0) before each step's entry read), LDS waits
(lgkmcnt(0)), the rest of the steps (arithmetic) -- plus the spread of wave start / end times across the launch
(realtime, so comparable across CUs) and the waves per SIMD that were live.
usage: python tools/comb_stamps.py build/ab/libpbft_stamps.so [sizes...]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    lib_path = sys.argv[1]
    sizes = [int(x) for x in sys.argv[2:]] or [131072, 1 << 20]
    os.environ["PBFT_VERIFY_LIB"] = os.path.abspath(lib_path)  # read by pbft_amd._lib at import
    import torch
    import bench
    torch.cuda.set_device(0)
    from pbft_amd import GpuBatchVerifier, _lib
    lib = _lib.load()
    assert os.path.samefile(lib._name, lib_path), lib._name
    lib.pbft_debug_comb_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    seeds = bench.key_seeds(256)
    msg, key_idx = bench.envelopes(1, 2048, 256)
    v = GpuBatchVerifier(0)
    R, S, pub = v.sign(seeds, key_idx, msg, 85)
    assert v.set_keys(pub).all()
    dev = torch.device("cuda", 0)
    d = bench.to_device(torch, dev, R, S, key_idx, msg)
    st = torch.cuda.Stream(dev)
    for n in sizes:
        for _ in range(30):  # warm: the clock settles under load
            v.verify_device(d["R"].data_ptr(), d["S"].data_ptr(), d["K"].data_ptr(), d["M"].data_ptr(), 85, 85, n,
                            d["B"].data_ptr(), st.cuda_stream)
        st.synchronize()
        waves = (n + 63) // 64
        buf = np.zeros((min(waves, 16384), 8), np.uint64)
        assert lib.pbft_debug_comb_stamps(buf.ctypes.data, len(buf)) == 0
        b = buf.astype(np.float64)
        life = b[:, 4] - b[:, 0]
        rt = (b[:, 5] - b[:, 1])
        clk = np.median(life / np.maximum(rt, 1)) * 0.1  # GHz (realtime ticks at 100 MHz)
        hash_ = b[:, 2] - b[:, 0]
        wait = b[:, 3]
        lgkm = b[:, 6]
        rest = life - hash_ - wait - lgkm
        t0 = b[:, 1].min()
        start = (b[:, 1] - t0) / 100.0  # us
        end = (b[:, 5] - t0) / 100.0
        hw = (buf[:, 7] & np.uint64(0xFFFFFFFF)).astype(np.int64)
        xcc = ((buf[:, 7] >> np.uint64(32)) & np.uint64(0xF)).astype(np.int64)
        simd = (hw >> 4) & 3
        cu = (hw >> 8) & 15
        sh = (hw >> 12) & 1
        se = (hw >> 13) & 3
        sid = (((xcc * 4 + se) * 2 + sh) * 16 + cu) * 4 + simd      # a SIMD of the chip
        cuid = sid >> 2
        _, inv_s, cnt_s = np.unique(sid, return_inverse=True, return_counts=True)
        _, inv_c, cnt_c = np.unique(cuid, return_inverse=True, return_counts=True)
        per_simd = cnt_s[inv_s]
        print(f"  placement: {len(cnt_c)} CUs, {len(cnt_s)} SIMDs used; waves per CU "
              + " ".join(f"{k}:{int((cnt_c == k).sum())}" for k in sorted(set(cnt_c.tolist())))
              + "; waves per SIMD " + " ".join(f"{k}:{int((cnt_s == k).sum())}" for k in sorted(set(cnt_s.tolist()))))
        for k in sorted(set(per_simd.tolist())):
            m = per_simd == k
            print(f"    waves on a SIMD shared by {k}: {int(m.sum())} waves, lifetime mean {life[m].mean():.0f} cyc, "
                  f"end mean {((b[m, 5] - b[:, 1].min()) / 100).mean():.1f} us")
        # waves live at each moment: sample at 200 points of the launch
        ts = np.linspace(0, end.max(), 200)
        live = np.array([((start <= t) & (end > t)).sum() for t in ts])
        print(f"== {n} signatures, {waves} waves: in-kernel clock {clk:.3f} GHz, launch span {end.max():.1f} us "
              f"(first wave end {end.min():.1f} us, last wave start {start.max():.1f} us)")
        for name, x in (("lifetime", life), ("hash+recode", hash_), ("gather vmcnt wait", wait),
                        ("LDS lgkmcnt wait", lgkm), ("steps other", rest)):
            print(f"  {name:18s} mean {x.mean():9.0f} cyc  p10 {np.percentile(x, 10):9.0f}  p90 "
                  f"{np.percentile(x, 90):9.0f}  ({100 * x.mean() / life.mean():5.1f} % of lifetime)")
        print(f"  wave start us: p0 {start.min():.1f} p50 {np.median(start):.1f} p90 {np.percentile(start, 90):.1f} "
              f"max {start.max():.1f}; end us: min {end.min():.1f} p10 {np.percentile(end, 10):.1f} p50 "
              f"{np.median(end):.1f} p90 {np.percentile(end, 90):.1f} max {end.max():.1f}")
        print(f"  live waves over the launch (200 samples): max {live.max()}, mean {live.mean():.0f} "
              f"(= {live.mean() / 1024:.2f} per SIMD), quartiles of time: "
              + " ".join(f"{live[i * 50:(i + 1) * 50].mean():.0f}" for i in range(4)))
    v.close()


if __name__ == "__main__":
    main()
