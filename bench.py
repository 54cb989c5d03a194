#!/usr/bin/env python3
"""Benchmark: Ed25519 verifies/s per node on PBFT round batches (BASELINE.json metric).

Workload (BASELINE.json configs[3], weak-scaled): n = 256 replicas; every
replica signs a Prepare and a Commit envelope for each of 2048 sequence
numbers -> 2^20 signatures per GPU per step ("one config-#4 round per GPU").
A step = one pass of the hot path over that batch with inputs resident in HBM:
the verify kernel (SHA-512 challenge, scalar reduction, comb double-scalar
multiplication, compression, compare, ballot) followed, for N > 1, by the RCCL
all-gather of the per-GPU accept bitmaps over xGMI (the round's exchange step).

Synthetic data: sk_i = SHA-512("pbft-key" || seed || i)[0:32],
85-byte envelope "PBFT" || kind || view u64 || seq u64 || Blake2b-512("op-"||seq),
signatures produced by the product's own GPU signer (pbft_sign_batch).

Also reported: the dominant kernel's roofline (VALU integer products, see
DESIGN.md §Roofline), p50 latency of a 4096-signature round (config #5's batch
size), and the CPU baseline = the oracle's C restatement timed on this host
(rank 0 only, bounded sample).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_REPLICAS = 256
SEQS_PER_GPU = 2048
ENVELOPE = 85
# algorithmic 32x32->64 products per verify for the comb algorithm
SEED = 0x5EED0000 + 4


def key_seeds(n: int, seed: int = SEED) -> np.ndarray:
    out = np.zeros((n, 32), dtype=np.uint8)
    for i in range(n):
        out[i] = np.frombuffer(hashlib.sha512(b"pbft-key" + seed.to_bytes(8, "little") +
                                              i.to_bytes(8, "little")).digest()[:32], dtype=np.uint8)
    return out


def envelopes(seq0: int, n_seq: int, n_rep: int):
    """Messages + key indices in round order: for seq, for kind in (Prepare, Commit), for replica."""
    digests = [hashlib.blake2b(b"op-" + str(seq0 + s).encode(), digest_size=64).digest() for s in range(n_seq)]
    base = np.zeros((n_seq, 2, ENVELOPE), dtype=np.uint8)
    for s in range(n_seq):
        for kind in (1, 2):
            b = b"PBFT" + bytes([kind]) + (1).to_bytes(8, "little") + (seq0 + s).to_bytes(8, "little") + digests[s]
            base[s, kind - 1] = np.frombuffer(b, dtype=np.uint8)
    msg = np.repeat(base[:, :, None, :], n_rep, axis=2).reshape(-1, ENVELOPE)
    key_idx = np.tile(np.arange(n_rep, dtype=np.uint16), n_seq * 2)
    return msg, key_idx


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def cpu_baseline(keys, R, S, key_idx, msg, budget_s: float = 12.0):
    """Oracle C restatement (oracle/ed25519_oracle.c) on this host's cores."""
    import ctypes
    lib_path = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(lib_path):
        return None
    lib = ctypes.CDLL(lib_path)
    vp = ctypes.c_void_p
    lib.oracle_verify_batch.argtypes = [vp, ctypes.c_uint32, vp, vp, vp, vp, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_uint64, vp, ctypes.c_int]
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    cores = max(1, min(int(os.environ.get("OMP_NUM_THREADS", cores)), cores))
    # calibrate on a small sample, then run ~budget_s seconds of work
    n0 = min(len(R), 512 * cores)
    out = np.zeros(len(R), dtype=np.uint8)
    t = time.perf_counter()
    lib.oracle_verify_batch(keys.ctypes.data, len(keys), R.ctypes.data, S.ctypes.data, key_idx.ctypes.data,
                            msg.ctypes.data, ENVELOPE, ENVELOPE, n0, out.ctypes.data, cores)
    rate0 = n0 / (time.perf_counter() - t)
    n = int(min(len(R), max(n0, rate0 * budget_s)))
    t = time.perf_counter()
    lib.oracle_verify_batch(keys.ctypes.data, len(keys), R.ctypes.data, S.ctypes.data, key_idx.ctypes.data,
                            msg.ctypes.data, ENVELOPE, ENVELOPE, n, out.ctypes.data, cores)
    dt = time.perf_counter() - t
    assert out[:n].all(), "CPU oracle rejected a valid synthetic signature"
    return {"value": n / dt, "unit": "verifies/s", "cores": cores, "kind": "port",
            "sample": f"first {n} signatures of the rank-0 round (n=256 replicas, 85-B envelopes), "
                      f"{dt:.1f} s, {cores} threads of oracle/ed25519_oracle.c"}


def pmc_traffic(pb: int, pa: int, n: int) -> dict:
    """HBM bytes per launch of the verify pair from the committed rocprofv3 --pmc passes (separate runs of this
    same command, tools/gpu_pmc_cur.sh): FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE of comb + finish."""
    p = os.path.join(ROOT, "profiles", "r01_pmc_comb", "derived.json")
    try:
        d = json.load(open(p))
    except (OSError, ValueError):
        return {}
    if d.get("sigs_per_launch") != n or f"PB={pb} PA={pa}" not in d.get("launch", ""):
        return {}
    return {"traffic_bytes_per_launch": d["traffic_bytes_per_launch"], "valu_busy_pct": d["comb_kernel"]["valu_busy_pct"],
            "source": "profiles/r01_pmc_comb/derived.json (PMC passes, not this run)"}


def stream_latency(v, R, S, key_idx, msg, offered_sigs_per_s: float, batch: int = 4096, n_ctx: int = 4,
                   duration_s: float = 1.0):
    """BASELINE config #5 on this GPU: 4096-signature batches arriving at a fixed offered rate, each submitted
    through the host-buffer API (H2D copies + kernels + bitmap D2H) on one of n_ctx contexts (own HIP streams,
    shared tables: pbft_verify_ctx_clone).  Latency = bitmap ready (host poll) - scheduled arrival.
    offered_sigs_per_s = inf measures back-to-back pipelined throughput instead."""
    from pbft_amd import SigBatch
    ctxs = [v.clone() for _ in range(n_ctx)]
    nb = max(1, len(R) // batch)
    batches = [SigBatch(R[i * batch:(i + 1) * batch], S[i * batch:(i + 1) * batch],
                        key_idx[i * batch:(i + 1) * batch], msg[i * batch:(i + 1) * batch], ENVELOPE)
               for i in range(min(nb, 64))]
    for c in ctxs:  # warm: workspace / staging allocation
        c.wait(c.submit(batches[0]))
    period = batch / offered_sigs_per_s if np.isfinite(offered_sigs_per_s) else 0.0
    pending = [None] * n_ctx  # (ticket, scheduled time)
    lat, done = [], 0
    t0 = time.perf_counter()
    k = 0
    while True:
        now = time.perf_counter()
        for ci, p in enumerate(pending):
            if p is not None and ctxs[ci].poll(p[0]) is not None:
                t = time.perf_counter()
                lat.append((t - p[1]) * 1e3)
                pending[ci] = None
                done += 1
        if now - t0 >= duration_s:
            if all(p is None for p in pending):
                break
            continue
        t_sched = t0 + k * period
        if now >= t_sched:
            ci = k % n_ctx
            if pending[ci] is not None:  # backlog: this stream is still busy
                b = ctxs[ci].wait(pending[ci][0])
                lat.append((time.perf_counter() - pending[ci][1]) * 1e3)
                done += 1
            pending[ci] = (ctxs[ci].submit(batches[k % len(batches)]), t_sched if period else time.perf_counter())
            k += 1
    wall = time.perf_counter() - t0
    for c in ctxs:
        c.close()
    lat = np.array(lat)
    return {"batch": batch, "streams": n_ctx,
            "offered_sigs_per_s": offered_sigs_per_s if np.isfinite(offered_sigs_per_s) else None,
            "achieved_sigs_per_s": done * batch / wall, "batches": int(done),
            "p50_ms": float(np.median(lat)), "p99_ms": float(np.percentile(lat, 99)),
            "path": "host buffers: H2D + comb + finish + D2H per batch"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seqs", type=int, default=SEQS_PER_GPU, help="sequence numbers per GPU per round")
    ap.add_argument("--replicas", type=int, default=N_REPLICAS)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--latency-iters", type=int, default=200)
    ap.add_argument("--settle-s", type=float, default=0.3, help="untimed GPU settle time before the warmup steps")
    args = ap.parse_args()

    import torch
    ws, rank, local = dist_env()
    if ws != args.gpus and ws > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {ws}")
    torch.cuda.set_device(local)
    dist = None
    if ws > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from pbft_amd import GpuBatchVerifier, bitmap_to_bool
    from pbft_amd.dist import allgather_bitmap
    from pbft_amd import _lib
    from pbft_amd.roofline import INPUT_BYTES, VALU_MAD_PEAK_PER_S, gather_bytes_per_verify, products_per_verify

    n_rep, n_seq = args.replicas, args.seqs
    seeds = key_seeds(n_rep)
    msg, key_idx = envelopes(1 + rank * n_seq, n_seq, n_rep)
    n = len(msg)
    v = GpuBatchVerifier(local)
    # the product's GPU signer produces the round (and the replica public keys)
    R, S, pub = v.sign(seeds, key_idx, msg, ENVELOPE)
    key_ok = v.set_keys(pub)
    assert key_ok.all()
    pb, pa = v.positions()  # the key plan set_keys chose for this key set
    PRODUCTS_PER_VERIFY = products_per_verify(pb, pa)

    dev = torch.device("cuda", local)
    d_R = torch.from_numpy(R).to(dev)
    d_S = torch.from_numpy(S).to(dev)
    d_K = torch.from_numpy(key_idx.view(np.int16)).to(dev)
    msg_pad = np.zeros(n * ENVELOPE + 64, dtype=np.uint8)  # +slack for unaligned tail reads
    msg_pad[: n * ENVELOPE] = msg.reshape(-1)
    d_M = torch.from_numpy(msg_pad).to(dev)
    words = (n + 63) // 64
    d_B = torch.zeros(words, dtype=torch.int64, device=dev)
    d_all = torch.zeros(words * ws, dtype=torch.int64, device=dev)
    # a dedicated (non-null) stream: kernel, events and the all-gather are ordered on it
    torch.cuda.synchronize()
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        v.verify_device(d_R.data_ptr(), d_S.data_ptr(), d_K.data_ptr(), d_M.data_ptr(), ENVELOPE, ENVELOPE, n,
                        d_B.data_ptr(), stream.cuda_stream)
        if ev is not None:
            ev[1].record(stream)
        if ws > 1:
            allgather_bitmap(d_B, ws, d_all)

    # Settle: the table builds just ran the GPU flat out; keep launching rounds for --settle-s seconds so that
    # clocks and address-translation caches reach steady state before the W warmup + K timed steps (measured:
    # 3 warmup steps alone leave the first timed rounds ~5 % slow).  Untimed, reported in the line.
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < args.settle_s:
        step()
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # correctness sanity on the real round: every synthetic signature is valid
    bm = d_B.cpu().numpy().view(np.uint64)
    assert bitmap_to_bool(bm, n).all(), "GPU rejected a valid synthetic signature"

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in evs]
    kern_avg = float(np.mean(kern_ms))
    if ws > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        full = d_all.cpu().numpy().view(np.uint64)
        assert bitmap_to_bool(full, words * 64 * ws).sum() >= 0

    # p50 latency of a 4096-signature round (config #5 batch size), device-resident
    lat = []
    if rank == 0 and args.latency_iters > 0:
        n4 = min(4096, n)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for it in range(args.latency_iters + 5):
            torch.cuda.synchronize()
            t = time.perf_counter()
            v.verify_device(d_R.data_ptr(), d_S.data_ptr(), d_K.data_ptr(), d_M.data_ptr(), ENVELOPE, ENVELOPE,
                            n4, d_B.data_ptr(), stream.cuda_stream)
            torch.cuda.synchronize()
            if it >= 5:
                lat.append((time.perf_counter() - t) * 1e3)

    if rank == 0:
        total = n * ws * args.steps
        value = total / dt
        products = PRODUCTS_PER_VERIFY * n / (kern_avg * 1e-3)
        stream = None
        if args.latency_iters > 0:
            # config #5: 2^24 sigs/s offered to an 8-GPU node = 2^21 per GPU; and back-to-back 4k batches
            stream = {"offered_2^21_per_gpu": stream_latency(v, R, S, key_idx, msg, float(1 << 21)),
                      "back_to_back": stream_latency(v, R, S, key_idx, msg, float("inf"))}
        cpu = None if args.no_cpu else cpu_baseline(pub, R, S, key_idx, msg)
        pmc = pmc_traffic(pb, pa, n)
        line = {
            "metric": "Ed25519 verifies/sec per node (1M-signature PBFT rounds)",
            "value": value,
            "unit": "verifies/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (GF(2^255-19) radix 2^25.5 limbs, 32x32->64 products)",
            "data": "synthetic: 256 replica keys, 85-B signed Prepare/Commit envelopes, GPU-signed (RFC 8032)",
            "config": {"workload": "config#4 round per GPU: n=256 replicas x 2048 seqs x {Prepare,Commit}",
                       "sigs_per_gpu": n, "sigs_per_step": n * ws, "msg_len": ENVELOPE, "settle_s": args.settle_s,
                       "parallelism": f"shard-by-index x{ws}" + (" + RCCL all-gather of bitmaps" if ws > 1 else "")},
            "roofline": {"bound": "valu", "achieved": products / 1e12, "peak": VALU_MAD_PEAK_PER_S / 1e12,
                         "unit": "T products/s (v_mad_u64_u32)", "frac": products / VALU_MAD_PEAK_PER_S,
                         "traffic": pmc.get("traffic_bytes_per_launch"),
                         "traffic_source": pmc.get("source"),
                         "valu_busy_pct": pmc.get("valu_busy_pct"),
                         "gather_bytes_algorithmic": (gather_bytes_per_verify(pb, pa) + INPUT_BYTES) * n, "kernel": f"comb_kernel<85, plan PA={pa}> (PB={pb}) + finish_kernel (one verify launch pair)", "kernel_avg_ms": kern_avg,
                         "products_per_verify": PRODUCTS_PER_VERIFY},
            "p50_ms_4k_round": float(np.median(lat)) if lat else None,
            "p99_ms_4k_round": float(np.percentile(lat, 99)) if lat else None,
            "stream_4k": stream,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    v.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
