#!/usr/bin/env python3
"""Benchmark: Ed25519 verifies/s per node on 1M-signature PBFT rounds (BASELINE.json metric).

Workload (BASELINE.json configs[3]): ONE round of n = 256 replicas x 2048
sequence numbers x {Prepare, Commit} = 2^20 signed 85-byte envelopes, sharded
by signature index over the N GPUs of the node (pbft_amd.dist.shard_bounds:
contiguous, 64-aligned).  A step = every rank verifies its shard with inputs
resident in HBM (verify kernels: SHA-512 challenge, scalar reduction, comb
double-scalar multiplication, compression, compare, ballot), then the per-rank
bitmaps are combined with one RCCL all-gather over xGMI into the round's
bitmap.  value = 2^20 x steps / max-over-ranks wall time (strong scaling: the
round is fixed, more GPUs share it).  0.1 % of the round's signatures are
corrupted (seeded positions): the assembled bitmap is checked against them.
A weak-scaling figure (every rank verifies a whole 2^20 round) is reported
beside it as `weak_scaling`.

Synthetic data: sk_i = SHA-512("pbft-key" || seed || i)[0:32],
85-byte envelope "PBFT" || kind || view u64 || seq u64 || Blake2b-512("op-"||seq),
signatures produced by the product's own GPU signer (pbft_sign_batch).

Rank 0 at N = 1 also reports: the dominant kernels' roofline, the 131k-signature
shard an 8-GPU node gives each GPU, the host-buffer (PCIe-inclusive) 2^20 round,
config #2 (n = 4, 1,024 pipelined requests = 8,192 signatures), p50 of a
4096-signature round and config #5 streaming, and two CPU baselines on this
host's cores: the oracle's C restatement ("port") and OpenSSL EVP_DigestVerify
(the SURVEY.md §8c substitute for ed25519-dalek).
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_REPLICAS = 256
SEQS = 2048
ENVELOPE = 85
SEED = 0x5EED0000 + 4
ADV_FRAC = 0.001


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


def corrupt(S: np.ndarray, frac: float, seed: int):
    """Flip one bit of s in a seeded `frac` of the signatures; returns the corrupted copy and the positions."""
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(len(S), size=max(1, int(len(S) * frac)), replace=False))
    S = S.copy()
    S[idx, rng.integers(0, 31, len(idx))] ^= np.uint8(4)
    return S, idx


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def host_cores() -> int:
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return max(1, min(int(os.environ.get("OMP_NUM_THREADS", cores)), cores))


def _cpu_lib(name: str, fn: str):
    path = os.path.join(ROOT, "oracle", name)
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    getattr(lib, fn).argtypes = [vp, ctypes.c_uint32, vp, vp, vp, vp, ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.c_uint64, vp, ctypes.c_int]
    return lib


def cpu_rate(fn, keys, R, S, key_idx, msg, budget_s: float, cores: int, expect=None):
    """Calibrate on a small sample, then time ~budget_s seconds of the same batch on `cores` threads."""
    out = np.zeros(len(R), dtype=np.uint8)
    args = lambda n: (keys.ctypes.data, len(keys), R.ctypes.data, S.ctypes.data, key_idx.ctypes.data,  # noqa: E731
                      msg.ctypes.data, ENVELOPE, ENVELOPE, n, out.ctypes.data, cores)
    n0 = min(len(R), 256 * cores)
    t = time.perf_counter()
    fn(*args(n0))
    rate0 = n0 / (time.perf_counter() - t)
    n = int(min(len(R), max(n0, rate0 * budget_s)))
    t = time.perf_counter()
    fn(*args(n))
    dt = time.perf_counter() - t
    if expect is not None:
        assert (out[:n].astype(bool) == expect[:n]).all(), "CPU baseline disagrees with the expected bits"
    return n / dt, n, dt


def cpu_baselines(keys, R, S, key_idx, msg, expect, budget_s: float = 10.0):
    cores = host_cores()
    res = {}
    o = _cpu_lib("liboracle.so", "oracle_verify_batch")
    if o is not None:
        v, n, dt = cpu_rate(o.oracle_verify_batch, keys, R, S, key_idx, msg, budget_s, cores, expect)
        res["port"] = {"value": v, "unit": "verifies/s", "cores": cores, "kind": "port",
                       "sample": f"first {n} signatures of the config-#4 round (n=256, 85-B envelopes, 0.1% "
                                 f"corrupted), {dt:.1f} s, {cores} threads of oracle/ed25519_oracle.c "
                                 f"(dalek verify_strict restatement)"}
    s = _cpu_lib("libossl_baseline.so", "ossl_verify_batch")
    if s is not None:
        s.ossl_version.restype = ctypes.c_char_p
        v, n, dt = cpu_rate(s.ossl_verify_batch, keys, R, S, key_idx, msg, budget_s, cores, expect)
        res["openssl"] = {"value": v, "unit": "verifies/s", "cores": cores, "kind": "openssl-substitute",
                          "sample": f"first {n} signatures of the config-#4 round, {dt:.1f} s, {cores} threads of "
                                    f"{s.ossl_version().decode()} EVP_DigestVerify (oracle/openssl_baseline.c; "
                                    f"SURVEY §8c substitute for ed25519-dalek verify_batch)"}
    return res


def pmc_traffic(pb: int, pa: int, n: int) -> dict:
    """HBM bytes per launch of the verify pair from the committed rocprofv3 --pmc passes (separate runs of this
    same command, tools/gpu_prof.sh): FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE of comb + finish."""
    for rel in ("r06/pmc_comb", "r05/pmc_comb", "r04/pmc_comb", "r03/pmc_comb", "r02_pmc_comb", "r01_pmc_comb"):
        p = os.path.join(ROOT, "profiles", rel, "derived.json")
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        if d.get("sigs_per_launch") != n or f"PB={pb} PA={pa}" not in d.get("launch", ""):
            continue
        return {"traffic_bytes_per_launch": d["traffic_bytes_per_launch"],
                "valu_busy_pct": d["comb_kernel"]["valu_busy_pct"],
                "valu_insts_per_sig": d.get("valu_insts_per_sig_total"),
                "valu_insts_per_sig_comb": d["comb_kernel"].get("valu_insts_per_sig"),
                "source": f"profiles/{rel}/derived.json (PMC passes, not this run)"}
    return {}


def shard_pmc(n: int) -> dict:
    """the shard's comb and finish duration and VALU busy from the committed rocprofv3 trace + PMC
    passes of this library at the shard size (tools/gpu_prof.sh with --seqs 256; profiles/r06/shard/derived.json)."""
    p = os.path.join(ROOT, "profiles", "r06", "shard", "derived.json")
    try:
        d = json.load(open(p))
    except (OSError, ValueError):
        return {}
    if d.get("sigs_per_launch") != n:
        return {}
    out = {"source": "profiles/r06/shard/derived.json (rocprofv3 trace + PMC passes, not this run)"}
    for k in ("comb_kernel", "finish_kernel"):
        e = d.get(k, {})
        out[k] = {"us": (e.get("avg_ns") or 0) / 1e3 or None, "valu_busy_pct": e.get("valu_busy_pct"),
                  "valu_insts_per_sig": e.get("valu_insts_per_sig")}
    return out


def stream_latency(v, R, S, key_idx, msg, offered_sigs_per_s: float, batch: int = 4096, n_ctx: int = 4,
                   duration_s: float = 1.0, pinned: bool = True):
    """BASELINE config #5 on this GPU: 4096-signature batches arriving at a fixed offered rate, each submitted
    through the host-buffer API (H2D copies + kernels + bitmap D2H) on one of n_ctx contexts (own HIP streams,
    shared tables: pbft_verify_ctx_clone).  Latency = bitmap ready (host poll) - scheduled arrival.
    offered_sigs_per_s = inf measures back-to-back pipelined throughput instead.  pinned: the batches live in
    pinned host memory (DMA'd in place); else pageable numpy arrays (the library copies them into its pinned
    staging inside the submit)."""
    from pbft_amd import SigBatch
    ctxs = [v.clone() for _ in range(n_ctx)]
    if pinned:
        import torch
        pin = lambda a: torch.from_numpy(np.ascontiguousarray(a)).pin_memory().numpy()  # noqa: E731
        m = min(len(R), 64 * batch)
        R, S, key_idx, msg = pin(R[:m]), pin(S[:m]), pin(key_idx[:m]), pin(msg[:m])
    nb = max(1, len(R) // batch)
    batches = [SigBatch(R[i * batch:(i + 1) * batch], S[i * batch:(i + 1) * batch],
                        key_idx[i * batch:(i + 1) * batch], msg[i * batch:(i + 1) * batch], ENVELOPE)
               for i in range(min(nb, 64))]
    for c in ctxs:  # warm: workspace / staging allocation
        c.wait(c.submit(batches[0]))
    period = batch / offered_sigs_per_s if np.isfinite(offered_sigs_per_s) else 0.0
    pending = [None] * n_ctx  # (ticket, scheduled time, submit start, submit end)
    lat, done = [], 0
    rec = []  # per batch: (latency, queue delay, submit, wait, largest gap between polls while waiting) in ms
    gap_since = [0.0] * n_ctx  # per context: the largest gap between consecutive poll passes while it was pending
    last_pass = time.perf_counter()
    import gc
    gc.collect()
    gc.disable()  # no collector pause inside the timed loop (a host-side tail, not the verifier's)
    t0 = time.perf_counter()
    k = 0
    while True:
        now = time.perf_counter()
        gap = now - last_pass
        last_pass = now
        for ci, p in enumerate(pending):
            if p is not None:
                gap_since[ci] = max(gap_since[ci], gap)
            if p is not None and ctxs[ci].poll(p[0]) is not None:
                t = time.perf_counter()
                lat.append((t - p[1]) * 1e3)
                rec.append(((t - p[1]) * 1e3, (p[2] - p[1]) * 1e3, (p[3] - p[2]) * 1e3, (t - p[3]) * 1e3,
                            gap_since[ci] * 1e3))
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
                p = pending[ci]
                ctxs[ci].wait(p[0])
                t = time.perf_counter()
                lat.append((t - p[1]) * 1e3)
                rec.append(((t - p[1]) * 1e3, (p[2] - p[1]) * 1e3, (p[3] - p[2]) * 1e3, (t - p[3]) * 1e3,
                            gap_since[ci] * 1e3))
                done += 1
            ts = time.perf_counter()
            tk = ctxs[ci].submit(batches[k % len(batches)])
            pending[ci] = (tk, t_sched if period else ts, ts, time.perf_counter())
            gap_since[ci] = 0.0
            k += 1
    wall = time.perf_counter() - t0
    gc.enable()
    for c in ctxs:
        c.close()
    lat = np.array(lat)
    worst = max(rec, key=lambda x: x[0]) if rec else (0, 0, 0, 0, 0)
    # the slowest batch's phases: queue (its scheduled arrival -> the submit call: the loop was busy elsewhere),
    # submit (the host call: staging / import kernel / launches), wait (submit return -> the poll that saw its bitmap:
    # GPU time + wake-up), and the largest gap between two poll passes meanwhile (> ~0.1 ms: this Python thread was
    # descheduled, a host-side stall, not the verifier)
    max_batch = dict(zip(("latency_ms", "queue_ms", "submit_ms", "wait_ms", "max_poll_gap_ms"), map(float, worst)))
    return {"batch": batch, "streams": n_ctx, "max_batch": max_batch,
            "offered_sigs_per_s": offered_sigs_per_s if np.isfinite(offered_sigs_per_s) else None,
            "achieved_sigs_per_s": done * batch / wall, "batches": int(done),
            "p50_ms": float(np.median(lat)), "p99_ms": float(np.percentile(lat, 99)),
            "p999_ms": float(np.percentile(lat, 99.9)), "max_ms": float(lat.max()),
            "inputs": "pinned host memory" if pinned else "pageable host memory (copied into the pinned staging)",
            "path": "host buffers: H2D + verify kernels + D2H per batch"}


def time_device(v, stream, d, n, iters, torch):
    """Average ms of `iters` back-to-back device-resident launches over the first n signatures (HIP events on the
    launch stream), and the wall ms per launch."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    e0.record(stream)
    for _ in range(iters):
        v.verify_device(d["R"].data_ptr(), d["S"].data_ptr(), d["K"].data_ptr(), d["M"].data_ptr(), ENVELOPE,
                        ENVELOPE, n, d["B"].data_ptr(), stream.cuda_stream)
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters, (time.perf_counter() - t) * 1e3 / iters


def to_device(torch, dev, R, S, key_idx, msg):
    n = len(R)
    msg_pad = np.zeros(n * ENVELOPE + 64, dtype=np.uint8)  # + slack for unaligned tail reads
    msg_pad[: n * ENVELOPE] = msg.reshape(-1)
    return {"R": torch.from_numpy(np.ascontiguousarray(R)).to(dev),
            "S": torch.from_numpy(np.ascontiguousarray(S)).to(dev),
            "K": torch.from_numpy(np.ascontiguousarray(key_idx).view(np.int16)).to(dev),
            "M": torch.from_numpy(msg_pad).to(dev),
            "B": torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)}


def e2e_host_round(v, R, S, key_idx, msg, expect, torch, iters: int = 5):
    """PCIe-inclusive 2^20 round: pinned host buffers -> pbft_verify_batch (chunked H2D on a copy stream overlapping
    the verify kernels, bitmap D2H).  Returns verifies/s and ms per round (median of iters)."""
    from pbft_amd import SigBatch, bitmap_to_bool
    n = len(R)
    pin = lambda a: torch.from_numpy(np.ascontiguousarray(a)).pin_memory().numpy()  # noqa: E731
    b = SigBatch(pin(R), pin(S), pin(key_idx), pin(msg), ENVELOPE)
    bm = v.verify(b)  # warm (staging allocation)
    assert (bitmap_to_bool(bm, n) == expect).all(), "host-buffer path bitmap differs"
    ts = []
    for _ in range(iters):
        t = time.perf_counter()
        v.verify(b)
        ts.append(time.perf_counter() - t)
    ms = float(np.median(ts)) * 1e3
    return {"value": n / (ms * 1e-3), "unit": "verifies/s", "ms_per_round": ms, "sigs": n,
            "path": "pinned host buffers: H2D (2^18-signature chunks on a copy stream, overlapped) + verify kernels "
                    "+ bitmap D2H, pbft_verify_batch", "bytes_h2d_per_sig": 32 + 32 + 2 + ENVELOPE}


def e2e_votes_round(v, R, S, key_idx, msg, expect, torch, iters: int = 5):
    """PCIe-inclusive 2^20 round in the votes form (pbft_verify_votes): per signature R, S, key index and a 4-byte
    index into the round's 4,096 distinct envelopes (one per (seq, kind)), 70 B instead of 151 B over PCIe."""
    from pbft_amd import bitmap_to_bool
    env, inv = np.unique(msg, axis=0, return_inverse=True)
    ei = inv.reshape(-1).astype(np.uint32)
    pin = lambda a: torch.from_numpy(np.ascontiguousarray(a)).pin_memory().numpy()  # noqa: E731
    Rp, Sp, Kp, Ip, Ep = pin(R), pin(S), pin(key_idx), pin(ei), pin(env)
    bm = v.verify_votes(Rp, Sp, Kp, Ip, Ep)
    assert (bitmap_to_bool(bm, len(R)) == expect).all(), "votes path bitmap differs"
    ts = []
    for _ in range(iters):
        t = time.perf_counter()
        v.verify_votes(Rp, Sp, Kp, Ip, Ep)
        ts.append(time.perf_counter() - t)
    ms = float(np.median(ts)) * 1e3
    return {"value": len(R) / (ms * 1e-3), "unit": "verifies/s", "ms_per_round": ms, "sigs": len(R),
            "envelopes": len(env), "bytes_h2d_per_sig": 32 + 32 + 2 + 4,
            "path": "pinned host buffers: pbft_verify_votes (R, S, key index, envelope index per signature + the "
                    "round's envelope table), chunked H2D overlapped with the kernels, bitmap D2H"}


def votes_device_round(v, d, msg, expect, stream, torch, dev, iters: int = 50):
    """The same 2^20 round device-resident in the votes form (pbft_verify_votes_device): R, S, key index, envelope
    index per signature + the round's 4,096 envelopes, whose block-2 SHA-512 schedule is expanded once per envelope
    inside the call (sha512.h sha512_env_sched).  Labelled figure beside `value` (which is the per-signature
    message form of include/pbft_verify.h pbft_verify_batch_device)."""
    from pbft_amd import bitmap_to_bool
    env, inv = np.unique(msg, axis=0, return_inverse=True)
    ep = np.zeros(len(env) * ENVELOPE + 64, dtype=np.uint8)  # + slack for the aligned tail reads
    ep[: len(env) * ENVELOPE] = env.reshape(-1)
    dE = torch.from_numpy(ep).to(dev)
    dI = torch.from_numpy(inv.reshape(-1).astype(np.int32)).to(dev)
    n = len(msg)

    def run():
        v.verify_votes_device(d["R"].data_ptr(), d["S"].data_ptr(), d["K"].data_ptr(), dI.data_ptr(), dE.data_ptr(),
                              len(env), n, d["B"].data_ptr(), stream.cuda_stream)

    run()
    torch.cuda.synchronize()
    assert (bitmap_to_bool(d["B"].cpu().numpy().view(np.uint64), n) == expect).all(), "votes device bitmap differs"
    for _ in range(5):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(iters):
        run()
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    return {"value": n / (ms * 1e-3), "unit": "verifies/s", "ms_per_round": ms, "sigs": n, "envelopes": len(env),
            "path": "device-resident votes form: envelope-schedule kernel + comb + finish per call"}


def replica_round_leg(v, seeds, pub, R, S, key_idx, msg, expect, rounds: int = 9, n_ctx: int = 1, modes=None,
                      mode_env: str = "PBFT_REPLICA_DIRECT"):
    """config #4's round through the replica state machine (include/pbft_replica.h)
    on this GPU, the way a reference replica runs it, ingest included: ONE long-lived pbft_replica (n = 256; its
    windows are recycled from round to round, as a running replica's are) receives each round's 2048 signed
    PrePrepares and 2^20 Prepare / Commit votes (pbft_replica_push_many: the per-row checks and window inserts on
    the worker pool, each window's rows on one thread, every vote's 72-byte staged row written into the replica's
    pinned row arena as it is pushed, and the arena's verification launched in parts while the threads push: r05,
    VERDICT r04 item 6 -- before, the flush filled the context's staging from the windows, a second pass over every
    vote, and only then copied it), then ONE pbft_replica_flush_submit (adopts that batch) and
    pbft_replica_flush_poll from the loop until the bitmap is applied and the events are out.  Timed: push_many -> last poll (`value`), and submit -> last poll (`flush_*`).  Round r
    covers seqs r * 2048 + 1 .. (r + 1) * 2048 (every round re-signed on the GPU: new envelopes); its bitmap
    pattern is the headline round's.  n_ctx > 1: pbft_replica_create_multi over the context and n_ctx - 1 clones
    (each context stages, launches and returns its own slice of the batch; on a node they would
    be one context per GPU, each with its own PCIe link -- here they share this GPU and its link).  modes: values of
    an environment variable (mode_env, default PBFT_REPLICA_DIRECT) cycled round by round (an interleaved A/B in one
    process; medians per mode in `by_mode`)."""
    import ctypes
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from replica_sim import Event, Stats, lib
    L = lib()
    n_rep = len(pub)
    n = len(R)
    n_seq = n // (2 * n_rep)
    # bench round order: for seq, for kind (Prepare, Commit), for replica
    kind = np.tile(np.repeat(np.array([1, 2], np.uint8), n_rep), n_seq)
    signer = key_idx.astype(np.uint32)
    view = np.ones(n, np.uint64)
    primary = 1 % n_rep
    bad = ~expect
    res = {k: [] for k in ("push_ms", "submit_ms", "flush_ms", "total_ms", "polls", "apply_ms")}
    phases = []  # per timed round: the replica's own phase timings (pbft_replica_get_timings)
    ev = (Event * 16384)()
    rep = ctypes.c_void_p()
    clones = [v.clone() for _ in range(n_ctx - 1)]
    ctxs = (ctypes.c_void_p * n_ctx)(v._ctx.value, *[c._ctx.value for c in clones])
    assert L.pbft_replica_create_multi(ctxs, n_ctx, n_rep, 0, pub.tobytes(), ctypes.byref(rep)) == 0
    st_prev = Stats()
    warm = 2  # rounds 0 and 1 size the replica's two row arenas (pushes alternate between them) and its windows
    mode_of = []
    for r in range(rounds + warm):
        if modes:
            os.environ[mode_env] = modes[r % len(modes)]
        seq0 = 1 + r * n_seq
        m, _ = envelopes(seq0, n_seq, n_rep) if r else (msg, None)
        if r:
            Rr, Sr, _ = v.sign(seeds, key_idx, m, ENVELOPE)
            Sr[bad] = S[bad]  # the headline round's corrupted positions (its corrupted s values fail here too)
        else:
            Rr, Sr = R, S
        seq = np.repeat(np.arange(seq0, seq0 + n_seq, dtype=np.uint64), 2 * n_rep)
        digs = np.ascontiguousarray(m[:, 21:85])
        sigs = np.ascontiguousarray(np.concatenate([Rr, Sr], axis=1))
        pp_env = m[::2 * n_rep].copy()
        pp_env[:, 4] = 0  # kind 0: the PrePrepare envelope of each seq
        pR, pS, _ = v.sign(seeds, np.full(n_seq, primary, np.uint16), pp_env, ENVELOPE)
        ops = [b"op-" + str(q).encode() for q in range(seq0, seq0 + n_seq)]
        for q in range(n_seq):
            assert L.pbft_replica_on_pre_prepare(rep, primary, 1, seq0 + q, ops[q], len(ops[q]),
                                                 digs[2 * n_rep * q].tobytes(), pR[q].tobytes() + pS[q].tobytes(),
                                                 None) == 1
        qd = ctypes.c_uint64()
        rows, ne = ctypes.c_uint64(), ctypes.c_uint32()
        t = time.perf_counter()
        assert L.pbft_replica_push_many(rep, n, kind.ctypes.data, view.ctypes.data, seq.ctypes.data, digs.ctypes.data,
                                        signer.ctypes.data, sigs.ctypes.data, ctypes.byref(qd)) == 0 and qd.value == n
        t0 = time.perf_counter()
        assert L.pbft_replica_flush_submit(rep, 0, ctypes.byref(rows)) == 0
        t1 = time.perf_counter()
        polls = 0
        while True:
            rc = L.pbft_replica_flush_poll(rep, ev, len(ev), ctypes.byref(ne))
            assert rc >= 0
            if rc == 1:
                break
            polls += 1
        t2 = time.perf_counter()
        assert rows.value == n + n_seq
        st = Stats()
        L.pbft_replica_get_stats(rep, ctypes.byref(st))
        assert st.rejected_sig - st_prev.rejected_sig == int(bad.sum()) and st.batches - st_prev.batches == 1
        committed = sum(1 for e in ev[: ne.value] if e.kind == 2)
        assert committed == n_seq, committed
        if r >= warm:
            res["push_ms"].append((t0 - t) * 1e3)
            res["submit_ms"].append((t1 - t0) * 1e3)
            res["flush_ms"].append((t2 - t0) * 1e3)
            res["total_ms"].append((t2 - t) * 1e3)
            res["polls"].append(polls)
            res["apply_ms"].append((st.apply_ns - st_prev.apply_ns) * 1e-6)
            phases.append(replica_timings(L, rep))
            mode_of.append(modes[r % len(modes)] if modes else None)
        st_prev = st
    if modes:
        os.environ.pop(mode_env, None)
    L.pbft_replica_destroy(rep)
    for c in clones:
        c.close()
    med = {k: float(np.median(x)) for k, x in res.items()}
    worst = int(np.argmax(res["total_ms"]))  # the slowest round, with its phases
    max_round = {"total_ms": res["total_ms"][worst], "push_many_ms": res["push_ms"][worst],
                 "flush_ms": res["flush_ms"][worst], "phases": phases[worst]}
    by_mode = None
    if modes:
        by_mode = {m: {k: float(np.median([x for x, mm in zip(v_, mode_of) if mm == m])) for k, v_ in res.items()}
                   for m in sorted(set(modes))}
        for m in by_mode:
            tot = [x for x, mm in zip(res["total_ms"], mode_of) if mm == m]
            by_mode[m]["total_ms_mean"] = float(np.mean(tot))
            by_mode[m]["total_ms_max"] = float(np.max(tot))
            ph = [x for x, mm in zip(phases, mode_of) if mm == m]
            by_mode[m]["phases_median"] = {k: float(np.median([x[k] for x in ph])) for k in ph[0]} if ph else {}
    return {"value": n / (med["total_ms"] * 1e-3), "unit": "verifies/s", "ms_per_round": med["total_ms"],
            **({"by_mode": by_mode} if by_mode else {}),
            "ms_per_round_min_max": [float(np.min(res["total_ms"])), float(np.max(res["total_ms"]))],
            "ms_per_round_mean": float(np.mean(res["total_ms"])), "max_round": max_round,
            "push_many_ms": med["push_ms"], "flush_ms": med["flush_ms"],
            "flush_verifies_per_s": n / (med["flush_ms"] * 1e-3),
            "flush_submit_ms": med["submit_ms"], "apply_ms": med["apply_ms"],
            "gpu_wait_ms": max(0.0, med["flush_ms"] - med["submit_ms"] - med["apply_ms"]),  # (medians of separate series)
            "polls_while_running": int(med["polls"]), "sigs": n + n_seq, "rounds": rounds, "contexts": n_ctx,
            "path": "one long-lived pbft_replica: push_many (2^20 votes, each one's 72-B staged row written into "
                    "the replica's pinned row arena, the arena launched in 8 parts -- H2D + kernels -- as the worker "
                    "threads finish them; + 2048 PrePrepares via on_pre_prepare, untimed) -> flush_submit (adopts that "
                    "early batch; PBFT_REPLICA_EARLY=0: hands the arena over as it is, PBFT_REPLICA_DIRECT=0: fills "
                    "the context's staging instead) -> "
                    "flush_poll loop applying each chunk's rows as its bitmap words land, until 2048 COMMITTED_LOCAL "
                    "events are out; value = votes / (push_many + flush); H2D 72 B/sig + 4096 envelopes; apply_ms = "
                    "time inside flush_poll applying, gpu_wait_ms = the rest of the polling"}


TIMING_FIELDS = ("push_checks_ns", "push_windows_ns", "push_rows_ns", "submit_segs_ns", "submit_launch_ns", "wait_ns",
                 "apply_partial_ns", "apply_final_ns", "gc_ns", "polls", "early_pieces", "early_piece_ns",
                 "early_last_rows", "push_checks_end_min_ns", "push_rows_start_max_ns", "push_rows_end_min_ns")


def replica_timings(L, rep):
    """pbft_replica_get_timings of the last push_many / flush (include/pbft_replica.h), in ms (counts as they are)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from replica_sim import Timings
    tm = Timings()
    assert L.pbft_replica_get_timings(rep, ctypes.byref(tm)) == 0
    return {k.replace("_ns", "_ms"): (getattr(tm, k) * 1e-6 if k.endswith("_ns") else int(getattr(tm, k)))
            for k in TIMING_FIELDS}


def replica_ingress_leg(v, seeds, pub, S_bad, bad, n_seq: int, modes=None):
    """config #4's round delivered to ONE long-lived pbft_replica the way the reference's caller
    delivers it -- one message at a time on ONE thread (the swarm's poll loop -> Pbft::inject_node_event,
    /root/reference/src/behavior.rs:304, arms :340-412) -- then flush_submit -> flush_poll.
    The loops run natively (tools/ingress/ingress_driver.cpp) and time themselves around the calls into the product:
      push         one pbft_replica_push per vote, in arrival order;
      records_1    each of the 256 connections' byte stream of 160-B binary records (built untimed with
                   pbft_amd.wire.records_pack), the loop visiting the connections round-robin and handing ONE record
                   per visit to pbft_replica_push_records;
      records_64   the same, 64 records (10 KiB, one socket read's worth) per visit;
      json_1       each connection's UviBytes/JSON frames (pbft_amd.wire.encode_votes), one frame per visit to
                   pbft_replica_push_frames;
      json_64      the same, 64 frames (~22 KiB) per visit: the parse rate once a read's frames are consecutive;
    and json_decode_64: those visits' frames decoded only (pbft_wire_decode_json, no replica) -- the parse's share.
    Round-robin visits deliver the round in time order: for seq, for kind, every peer's vote.  The signed PrePrepares
    (on_pre_prepare, GPU digest) are delivered first, untimed.  With a flush behind it (the first rounds) the
    single-message path opens the arena as a batch in pieces on the GPU while the votes arrive (r06), so the flush is
    the last piece, the GPU's tail and the application.  Per mode: ingress votes/s (the loop alone), end to end
    ((ingress + flush)), and the replica's own phase timings of its slowest round (pbft_replica_get_timings)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from replica_sim import Event, Stats, lib
    from pbft_amd import wire
    from pbft_amd.native_build import INGRESS_LIB
    L = lib()
    D = ctypes.CDLL(INGRESS_LIB)
    vp = ctypes.c_void_p
    D.ingress_push.argtypes = [vp, ctypes.c_uint64, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    D.ingress_streams.argtypes = [vp, ctypes.c_int, ctypes.c_uint32, vp, vp, ctypes.c_uint32, vp, vp, vp, vp, vp]
    D.ingress_decode_only.argtypes = [ctypes.c_uint32, vp, vp, ctypes.c_uint32, vp, vp, vp]
    pmu_names = ("cycles", "instructions", "llc_references", "llc_misses", "l1d_read_misses", "dtlb_read_misses")
    pmu = (ctypes.c_uint64 * D.ingress_pmu_counters())()
    n_rep = len(pub)
    n = 2 * n_rep * n_seq
    modes = modes or [("push", 2, True), ("push", 3, False), ("records_1", 3, False), ("records_64", 2, False),
                      ("json_1", 1, False), ("json_64", 1, False)]
    primary = 1 % n_rep
    ev = (Event * 16384)()
    rep = ctypes.c_void_p()
    assert L.pbft_replica_create(v._ctx.value, n_rep, 0, pub.tobytes(), ctypes.byref(rep)) == 0
    kind = np.tile(np.repeat(np.array([1, 2], np.uint8), n_rep), n_seq)
    signer = np.tile(np.arange(n_rep, dtype=np.uint32), 2 * n_seq)
    view = np.ones(n, np.uint64)
    key_idx = signer.astype(np.uint16)
    res = {}
    st_prev = Stats()
    L.pbft_replica_get_stats(rep, ctypes.byref(st_prev))
    rnd = 0
    try:
        for mode, rounds, warm in modes:
            out = res.setdefault(mode, {"ingress_ms": [], "flush_ms": [], "timings": [], "pmu": []}) if not warm else None
            for _ in range(rounds):
                seq0 = 1 + rnd * n_seq  # (a replica of its own: its log starts at seq 1)
                rnd += 1
                m, _ = envelopes(seq0, n_seq, n_rep)
                Rr, Sr, _ = v.sign(seeds, key_idx, m, ENVELOPE)
                Sr[bad] = S_bad[bad]
                seq = np.repeat(np.arange(seq0, seq0 + n_seq, dtype=np.uint64), 2 * n_rep)
                digs = np.ascontiguousarray(m[:, 21:85])
                sigs = np.ascontiguousarray(np.concatenate([Rr, Sr], axis=1))
                pp_env = m[::2 * n_rep].copy()
                pp_env[:, 4] = 0
                pR, pS, _ = v.sign(seeds, np.full(n_seq, primary, np.uint16), pp_env, ENVELOPE)
                for q in range(n_seq):
                    op = b"op-" + str(seq0 + q).encode()
                    assert L.pbft_replica_on_pre_prepare(rep, primary, 1, seq0 + q, op, len(op),
                                                         digs[2 * n_rep * q].tobytes(),
                                                         pR[q].tobytes() + pS[q].tobytes(), None) == 1
                sec = ctypes.c_double()
                if mode == "push":
                    qd = ctypes.c_uint64()
                    assert D.ingress_push(rep, n, kind.ctypes.data, view.ctypes.data, seq.ctypes.data,
                                          digs.ctypes.data, signer.ctypes.data, sigs.ctypes.data, ctypes.byref(qd),
                                          ctypes.byref(sec), pmu) == 0 and qd.value == n
                else:
                    binary, per_visit = mode.startswith("records"), int(mode.split("_")[1])
                    streams = []
                    for c in range(n_rep):
                        sel = slice(c, None, n_rep)  # peer c's votes in (seq, kind) order
                        if binary:
                            streams.append(wire.records_pack(Rr[sel], Sr[sel], key_idx[sel], m[sel]).reshape(-1))
                        else:
                            streams.append(wire.encode_votes(kind[sel], view[sel], seq[sel], digs[sel], signer[sel],
                                                             sigs[sel]))
                    ptrs = (ctypes.c_void_p * n_rep)(*[s_.ctypes.data for s_ in streams])
                    lens = (ctypes.c_uint64 * n_rep)(*[len(s_) for s_ in streams])
                    pushed, dropped, calls = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
                    assert D.ingress_streams(rep, int(binary), n_rep, ptrs, lens, per_visit, ctypes.byref(pushed),
                                             ctypes.byref(dropped), ctypes.byref(calls), ctypes.byref(sec), pmu) == 0
                    assert pushed.value == n and dropped.value == 0, (pushed.value, dropped.value)
                    if not binary and per_visit > 1 and out is not None:  # the same visits, decoded only
                        frames, sec_d = ctypes.c_uint64(), ctypes.c_double()
                        pmu_d = (ctypes.c_uint64 * D.ingress_pmu_counters())()
                        assert D.ingress_decode_only(n_rep, ptrs, lens, per_visit, ctypes.byref(frames),
                                                     ctypes.byref(sec_d), pmu_d) == 0 and frames.value == n
                        out.setdefault("decode_ms", []).append(sec_d.value * 1e3)
                        out.setdefault("decode_pmu", []).append([int(x) for x in pmu_d])
                rows = ctypes.c_uint64()
                ne = ctypes.c_uint32()
                t0 = time.perf_counter()
                assert L.pbft_replica_flush_submit(rep, 0, ctypes.byref(rows)) == 0
                while True:
                    rc = L.pbft_replica_flush_poll(rep, ev, len(ev), ctypes.byref(ne))
                    assert rc >= 0
                    if rc == 1:
                        break
                t1 = time.perf_counter()
                assert rows.value == n + n_seq
                st = Stats()
                L.pbft_replica_get_stats(rep, ctypes.byref(st))
                assert st.rejected_sig - st_prev.rejected_sig == int(bad.sum()), "ingress round: rejected votes differ"
                assert sum(1 for e in ev[: ne.value] if e.kind == 2) == n_seq, "ingress round: not every seq committed"
                st_prev = st
                if out is not None:
                    out["ingress_ms"].append(sec.value * 1e3)
                    out["flush_ms"].append((t1 - t0) * 1e3)
                    out["timings"].append(replica_timings(L, rep))
                    out["pmu"].append([int(x) for x in pmu])
    finally:
        L.pbft_replica_destroy(rep)
    legs = {}
    for mode, o in res.items():
        ing, fl = np.array(o["ingress_ms"]), np.array(o["flush_ms"])
        tot = ing + fl
        worst = int(np.argmax(tot))
        pm = np.median(np.array(o["pmu"], dtype=np.float64), axis=0) if o["pmu"] else None
        host = None
        if pm is not None and pm[0] > 0:  # per vote, medians over the rounds (perf_event_open, user space)
            host = {k: float(v / n) for k, v in zip(pmu_names, pm)}
            host["ipc"] = float(pm[1] / pm[0])
            host["ghz"] = float(pm[0] / (np.median(ing) * 1e-3) / 1e9)
        if o.get("decode_ms"):
            dm = float(np.median(o["decode_ms"]))
            dp = np.median(np.array(o["decode_pmu"], dtype=np.float64), axis=0)
            dh = {k: float(v / n) for k, v in zip(pmu_names, dp)} if dp[0] > 0 else None
            if dh:
                dh["ipc"] = float(dp[1] / dp[0])
            legs[mode + "_decode_only"] = {"frames_per_s": n / (dm * 1e-3), "decode_ms": dm, "host_pmu_per_frame": dh}
        legs[mode] = {"ingress_votes_per_s": n / (np.median(ing) * 1e-3), "ingress_ms": float(np.median(ing)),
                      "host_pmu_per_vote": host,
                      "flush_ms": float(np.median(fl)), "flush_ms_max": float(fl.max()),
                      "end_to_end_votes_per_s": n / (np.median(tot) * 1e-3), "rounds": len(ing),
                      "max_round": {"ingress_ms": float(ing[worst]), "flush_ms": float(fl[worst]),
                                    "phases": o["timings"][worst]}}
    return {"votes": n, "prepreprares_untimed": n_seq, "thread": "one (the caller's)", "modes": legs,
            "path": "tools/ingress/ingress_driver.cpp loops -> pbft_replica_push / _push_records / _push_frames "
                    "(one message, or one 64-record read, per call; connections round-robin) -> flush_submit -> "
                    "flush_poll until every seq is COMMITTED_LOCAL; the single-message early batch launched in "
                    "2^16-row pieces while the votes arrive"}


def plan_legs(v, pub, d, n, stream, torch):
    """what a re-keying costs (set_keys of the n = 256 replica keys: decompress, small-order
    check, comb tables) and the 2^20 device-resident rate of every key plan a shared or smaller GPU falls back to
    (forced with PBFT_OPT_KEY_TABLE_BUDGET_MB).  Restores the default plan at the end."""
    import re
    info = v._lib.pbft_build_info().decode()
    pas = [int(x) for x in re.search(r"PA=([\d|]+)", info).group(1).split("|")]
    sizes = [int(x) for x in re.search(r"tabA/key=([\dB|]+)", info).group(1).replace("B", "").split("|")]
    per_key = dict(zip(pas, sizes))
    out = {}
    torch.cuda.synchronize()
    for name, budget in (("PLA_BIG_14", 100_000), ("PLA_MID_16", 20_000), ("PLA_SMALL_32", 1_000),
                         ("default", 0)):
        v.set_option(v.OPT_KEY_TABLE_BUDGET_MB, budget)
        t = time.perf_counter()
        assert v.set_keys(pub).all()
        ms_keys = (time.perf_counter() - t) * 1e3
        ks = v.key_stats()
        pb, pa = v.positions()
        time_device(v, stream, d, n, 3, torch)
        k, w = time_device(v, stream, d, n, 20, torch)
        out[name] = {"positions": [pb, pa], "steps": pb + pa, "set_keys_ms": ms_keys, "kernel_ms": k,
                     "verifies_per_s": n / (k * 1e-3), "key_tables_gb": per_key.get(pa, 0) * len(pub) / 1e9,
                     "phases_ms": {x: round(ks[x + "_ms"], 2) for x in ("free", "alloc", "build", "meminfo")},
                     "reused_allocation": bool(ks["reused"])}
    return out


def rekey_legs(v, pub, d, n, stream, torch, expect):
    """a re-key of the SAME n = 256 set (same plan: the table allocation is kept and rebuilt in
    place) and the replacement of ONE replica's key (pbft_verify_update_keys: only its tables are rebuilt, as when
    a peer is admitted later -- the reference's add_peer, src/behavior.rs:45-61); the round's bitmap is checked
    after each."""
    from pbft_amd import bitmap_to_bool
    out = {}
    torch.cuda.synchronize()
    t = time.perf_counter()
    assert v.set_keys(pub).all()
    out["rekey_ms"] = (time.perf_counter() - t) * 1e3
    ks = v.key_stats()
    out["rekey_phases_ms"] = {x: round(ks[x + "_ms"], 2) for x in ("free", "alloc", "build", "meminfo")}
    out["rekey_reused_allocation"] = bool(ks["reused"])
    times = []
    for slot in (17, 200, 17):
        t = time.perf_counter()
        assert v.update_keys([slot], pub[slot:slot + 1]).all()
        times.append((time.perf_counter() - t) * 1e3)
    out["update_one_key_ms"] = float(np.median(times))
    out["update_one_key_ms_all"] = times
    time_device(v, stream, d, n, 2, torch)
    got = bitmap_to_bool(d["B"].cpu().numpy().view(np.uint64), n)
    assert (got == expect[:n]).all(), "bitmap after re-key / update differs"
    return out


def shuffled_leg(v, d, n, stream, torch, dev, expect):
    """The headline round with its rows in a random order (every wave mixes envelopes and keys: block 2's SHA-512
    schedule per lane instead of the scalar unit's per-wave copy); VERDICT r02 item 9."""
    from pbft_amd import bitmap_to_bool
    perm = torch.from_numpy(np.random.default_rng(7).permutation(n)).to(dev)
    M = d["M"][: n * ENVELOPE].view(n, ENVELOPE)[perm].reshape(-1)
    ds = {"R": d["R"][perm].contiguous(), "S": d["S"][perm].contiguous(), "K": d["K"][perm].contiguous(),
          "M": torch.cat([M, torch.zeros(64, dtype=M.dtype, device=dev)]), "B": torch.zeros_like(d["B"])}
    time_device(v, stream, ds, n, 2, torch)
    got = bitmap_to_bool(ds["B"].cpu().numpy().view(np.uint64), n)
    assert (got == expect[perm.cpu().numpy()]).all(), "shuffled round bitmap differs"
    k, w = time_device(v, stream, ds, n, 20, torch)
    return {"kernel_ms": k, "verifies_per_s": n / (k * 1e-3),
            "note": "same 2^20 round, rows randomly permuted (device-resident)"}


def config2_leg(v, torch, dev, stream, cpu: bool, iters: int = 200):
    """BASELINE configs[1]: n = 4 replicas, 1,024 pipelined requests -> 8,192 signatures per window batch, one GPU
    (device-resident p50 and host-buffer p50) vs the CPU baselines on the same batch."""
    from pbft_amd import SigBatch, bitmap_to_bool
    c = v.clone()
    try:
        seeds = key_seeds(4, 0x5EED0000 + 2)
        msg, key_idx = envelopes(1, 1024, 4)
        R, S, pub = c.sign(seeds, key_idx, msg, ENVELOPE)
        assert c.set_keys(pub).all()
        d = to_device(torch, dev, R, S, key_idx, msg)
        lat = []
        for it in range(iters + 5):
            torch.cuda.synchronize()
            t = time.perf_counter()
            c.verify_device(d["R"].data_ptr(), d["S"].data_ptr(), d["K"].data_ptr(), d["M"].data_ptr(), ENVELOPE,
                            ENVELOPE, len(R), d["B"].data_ptr(), stream.cuda_stream)
            torch.cuda.synchronize()
            if it >= 5:
                lat.append((time.perf_counter() - t) * 1e3)
        assert bitmap_to_bool(d["B"].cpu().numpy().view(np.uint64), len(R)).all()
        host = []
        b = SigBatch(R, S, key_idx, msg, ENVELOPE)
        for it in range(min(iters, 100) + 3):
            t = time.perf_counter()
            bm = c.verify(b)
            if it >= 3:
                host.append((time.perf_counter() - t) * 1e3)
        assert bitmap_to_bool(bm, len(R)).all()
        out = {"sigs": len(R), "replicas": 4, "requests": 1024,
               "device_p50_ms": float(np.median(lat)), "device_verifies_per_s": len(R) / (np.median(lat) * 1e-3),
               "host_buffer_p50_ms": float(np.median(host))}
        if cpu:
            cores = host_cores()
            for name, lib, fn in (("cpu_port", "liboracle.so", "oracle_verify_batch"),
                                  ("cpu_openssl", "libossl_baseline.so", "ossl_verify_batch")):
                L = _cpu_lib(lib, fn)
                if L is not None:
                    rate, n, dt = cpu_rate(getattr(L, fn), pub, R, S, key_idx, msg, 2.0, cores,
                                           np.ones(len(R), bool))
                    out[name] = {"verifies_per_s": rate, "window_ms": len(R) / rate * 1e3, "cores": cores}
        return out
    finally:
        c.close()


L_ORDER = 2**252 + 27742317777372353535851937790883648493  # the group order L (RFC 8032)


def adversarial_round(R, S, frac: float, seed: int):
    """config #3's adversarial share: a seeded `frac` of the signatures made invalid in three ways, a third each --
    one bit of s flipped, s replaced by s + L (non-canonical: verify_strict rejects s >= L), one bit of R flipped.
    Returns the corrupted copies and the expected bits."""
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(len(S), size=max(3, int(len(S) * frac)), replace=False))
    R, S = R.copy(), S.copy()
    a, b, c = np.array_split(idx, 3)
    S[a, rng.integers(0, 31, len(a))] ^= np.uint8(4)
    for i in b:
        S[i] = np.frombuffer((int.from_bytes(S[i].tobytes(), "little") + L_ORDER).to_bytes(32, "little"), np.uint8)
    R[c, rng.integers(0, 31, len(c))] ^= np.uint8(2)
    expect = np.ones(len(R), bool)
    expect[idx] = False
    return R, S, expect


def config3_leg(v, torch, dev, stream, cpu: bool, iters: int = 100):
    """BASELINE configs[2]: n = 64 replicas (f = 21), one 2^16-signature round batch (512 seqs x {Prepare, Commit} x
    64) with 1 % adversarial signatures (flipped s, non-canonical s + L, flipped R), one GPU: device-resident p50 and
    throughput, the bitmap checked, and the CPU baselines on the same batch."""
    from pbft_amd import bitmap_to_bool
    c = v.clone()
    try:
        seeds = key_seeds(64, 0x5EED0000 + 3)
        msg, key_idx = envelopes(1, 512, 64)
        R0, S0, pub = c.sign(seeds, key_idx, msg, ENVELOPE)
        R, S, expect = adversarial_round(R0, S0, 0.01, 0x5EED0000 + 3)
        assert c.set_keys(pub).all()
        d = to_device(torch, dev, R, S, key_idx, msg)

        def p50():
            lat = []
            d["B"].zero_()
            for it in range(iters + 5):
                torch.cuda.synchronize()
                t = time.perf_counter()
                c.verify_device(d["R"].data_ptr(), d["S"].data_ptr(), d["K"].data_ptr(), d["M"].data_ptr(), ENVELOPE,
                                ENVELOPE, len(R), d["B"].data_ptr(), stream.cuda_stream)
                torch.cuda.synchronize()
                if it >= 5:
                    lat.append((time.perf_counter() - t) * 1e3)
            got = bitmap_to_bool(d["B"].cpu().numpy().view(np.uint64), len(R))
            assert (got == expect).all(), "config #3 bitmap differs from the expected bits"
            return float(np.median(lat))
        m = p50()
        out = {"sigs": len(R), "replicas": 64, "adversarial": int((~expect).sum()),
               "device_p50_ms": m, "device_verifies_per_s": len(R) / (m * 1e-3),
               "comb": "comb_pair_kernel (two waves per 64 signatures, by batch size)"}
        # the single-wave comb on the same batch (PBFT_OPT_COMB_PAIR = 0), for the pair comb's gain (bitmap checked)
        try:
            c.set_option(c.OPT_COMB_PAIR, 0)
            out["device_p50_ms_single_wave_comb"] = p50()
        except Exception as e:  # a diagnostic beside the measured line; its failure is reported, not fatal
            out["single_wave_comb_error"] = repr(e)
        finally:
            c.set_option(c.OPT_COMB_PAIR, 2)
        if cpu:
            cores = host_cores()
            for name, lib, fn in (("cpu_port", "liboracle.so", "oracle_verify_batch"),
                                  ("cpu_openssl", "libossl_baseline.so", "ossl_verify_batch")):
                L = _cpu_lib(lib, fn)
                if L is not None:
                    rate, n, dt = cpu_rate(getattr(L, fn), pub, R, S, key_idx, msg, 2.0, cores, expect)
                    out[name] = {"verifies_per_s": rate, "round_ms": len(R) / rate * 1e3, "cores": cores}
        return out
    finally:
        c.close()


def c_abi_multi_round(verifiers, R, S, key_idx, msg, expect, torch, steps: int, warmup: int = 2):
    """the round sharded over G GPUs of THIS process through the C ABI's single-process form
    (include/pbft_verify.h pbft_multi_create -> ncclCommInitAll over the contexts' devices;
    pbft_verify_batch_device_multi -> every context verifies its 64-aligned shard on its own stream, then ONE grouped
    in-place ncclAllGather of the bitmap words), the same shard layout as the one-process-per-GPU default
    (pbft_amd.dist).  Every device's gathered round bitmap is checked against the expected bits.  Returns
    (verifies/s, ms per step, the assembled round bitmap of device 0 as bools)."""
    from pbft_amd import MultiGpu, bitmap_to_bool
    from pbft_amd.dist import assemble, shard_bounds, shard_words
    G = len(verifiers)
    n_total = len(R)
    wpr = shard_words(n_total, G)
    devs, ns = [], []
    for r, v in enumerate(verifiers):
        lo, hi = shard_bounds(n_total, r, G)
        dev = torch.device("cuda", v.device)
        d = to_device(torch, dev, R[lo:hi], S[lo:hi], key_idx[lo:hi], msg[lo:hi])
        d["B"] = torch.zeros(wpr * G, dtype=torch.int64, device=dev)
        devs.append(d)
        ns.append(hi - lo)
    m = MultiGpu(verifiers)
    try:
        def step():
            m.verify_device([d["R"].data_ptr() for d in devs], [d["S"].data_ptr() for d in devs],
                            [d["K"].data_ptr() for d in devs], [d["M"].data_ptr() for d in devs], ns, wpr,
                            [d["B"].data_ptr() for d in devs])
        for _ in range(warmup):
            step()
        m.sync()
        t = time.perf_counter()
        for _ in range(steps):
            step()
        m.sync()
        dt = time.perf_counter() - t
        got = None
        for d in devs:
            words = assemble(d["B"], n_total, G)
            b = bitmap_to_bool(words.cpu().numpy().view(np.uint64), n_total)
            assert (b == expect).all(), "C-ABI multi-GPU round bitmap differs from the expected bits"
            got = b if got is None else got
        return n_total * steps / dt, dt / steps * 1e3, got
    finally:
        m.close()


def single_process_main(args):
    """--single-process: ONE process drives every GPU it sees (or --gpus N of them) through the C ABI
    (c_abi_multi_round); prints the headline line like the default mode.  The default mode (one process per GPU,
    torch.distributed over RCCL) is what the N > 1 driver runs use."""
    import torch
    from pbft_amd import GpuBatchVerifier
    G = args.gpus if args.gpus > 0 else torch.cuda.device_count()
    G = min(G, torch.cuda.device_count())
    seeds = key_seeds(args.replicas)
    msg, key_idx = envelopes(1, args.seqs, args.replicas)
    vs = [GpuBatchVerifier(g) for g in range(G)]
    for v in vs:
        v.set_option(v.OPT_KERNEL_TIMING, 0)
    R, S_good, pub = vs[0].sign(seeds, key_idx, msg, ENVELOPE)
    S, bad = corrupt(S_good, ADV_FRAC, SEED)
    expect = np.ones(len(msg), bool)
    expect[bad] = False
    for v in vs:
        assert v.set_keys(pub).all()
    c_abi_multi_round(vs, R, S, key_idx, msg, expect, torch, 3, args.warmup)  # settle
    value, ms, _ = c_abi_multi_round(vs, R, S, key_idx, msg, expect, torch, args.steps, args.warmup)
    print(json.dumps({
        "metric": "Ed25519 verifies/sec per node (1M-signature PBFT rounds)", "value": value, "unit": "verifies/s",
        "n_gpus": G, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u32 (GF(2^255-19) radix 2^25.5 limbs, 32x32->64 products)",
        "data": "synthetic: 256 replica keys, 85-B signed Prepare/Commit envelopes, GPU-signed (RFC 8032), 0.1% of "
                "signatures corrupted (bitmap checked on every device)",
        "config": {"workload": "config#4: one round of n=256 replicas x 2048 seqs x {Prepare,Commit} = 2^20 "
                               "signatures, sharded by index over the GPUs", "sigs_per_step": len(msg),
                   "msg_len": ENVELOPE,
                   "parallelism": f"single process, C ABI: pbft_verify_batch_device_multi x{G} + in-place "
                                  f"ncclAllGather of the bitmap words"}}), flush=True)
    for v in vs:
        v.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--seqs", type=int, default=SEQS, help="sequence numbers in the round (2 x replicas x seqs sigs)")
    ap.add_argument("--replicas", type=int, default=N_REPLICAS)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="only the headline line (no side legs)")
    ap.add_argument("--replica-only", action="store_true",
                    help="diagnosis: the headline, then only the replica legs (r06: where the in-bench leg's time goes)")
    ap.add_argument("--latency-iters", type=int, default=200)
    ap.add_argument("--stream-s", type=float, default=20.0, help="config #5 offered-load leg duration (s)")
    ap.add_argument("--settle-s", type=float, default=1.0, help="untimed GPU settle time before the warmup steps")
    ap.add_argument("--sequential", action="store_true", help="force rounds in order on one stream (the default)")
    ap.add_argument("--pipeline", action="store_true",
                    help="pipeline rounds: finish + all-gather of round k on a second stream under round k+1's comb")
    ap.add_argument("--single-process", action="store_true",
                    help="one process drives --gpus GPUs through the C ABI (pbft_multi_create + "
                         "pbft_verify_batch_device_multi); default: one process per GPU over torch.distributed")
    args = ap.parse_args()
    if args.single_process:
        return single_process_main(args)

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
    from pbft_amd.dist import allgather_bitmap, round_bitmap, shard_bounds, shard_words
    from pbft_amd.roofline import (INPUT_BYTES, VALU_MAD_PEAK_PER_S, gather_bytes_per_verify, mad_peak_at,
                                   products_comb, products_per_verify)

    n_rep, n_seq = args.replicas, args.seqs
    seeds = key_seeds(n_rep)
    msg, key_idx = envelopes(1, n_seq, n_rep)
    n_total = len(msg)
    v = GpuBatchVerifier(local)
    # the bench times launches with its own HIP events on the launch stream: the library's per-launch timing
    # events (pbft_last_kernel_ms) are switched off, as a latency-bound caller would (PBFT_OPT_KERNEL_TIMING)
    v.set_option(v.OPT_KERNEL_TIMING, 0)
    # the product's GPU signer produces the round (and the replica public keys); every rank builds the same round
    R, S_good, pub = v.sign(seeds, key_idx, msg, ENVELOPE)
    S, bad = corrupt(S_good, ADV_FRAC, SEED)
    expect = np.ones(n_total, bool)
    expect[bad] = False
    t_keys = time.perf_counter()
    key_ok = v.set_keys(pub)
    set_keys_ms = (time.perf_counter() - t_keys) * 1e3  # n = 256: decompression, small-order check, comb tables
    ks0 = v.key_stats()
    set_keys_phases = {x: round(ks0[x + "_ms"], 2) for x in ("free", "alloc", "build", "meminfo")}
    assert key_ok.all()
    pb, pa = v.positions()  # the key plan set_keys chose for this key set

    dev = torch.device("cuda", local)
    lo, hi = shard_bounds(n_total, rank, ws)
    n = hi - lo
    d = to_device(torch, dev, R[lo:hi], S[lo:hi], key_idx[lo:hi], msg[lo:hi])
    per_words = shard_words(n_total, ws)
    d_local = torch.zeros(per_words, dtype=torch.int64, device=dev)   # this rank's bitmap words (padded)
    d_all = torch.zeros(per_words * ws, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    stream = torch.cuda.Stream(dev)      # comb kernels (and everything, --sequential)
    fin_stream = torch.cuda.Stream(dev)  # pipelined rounds: finish + bitmap all-gather of round k under comb of k+1
    torch.cuda.set_stream(stream)
    # --pipeline: round k's finish and bitmap all-gather (fin_stream) run under round k+1's comb kernel (stream).
    # Off by default: measured at N = 1 within 1 % of sequential on a 2^20 round and 15 % SLOWER on the 131k
    # shard of an 8-GPU node (0.246 vs 0.215 ms: the finish competes for the same VALUs and the cross-stream
    # events cost more than they hide), so rounds run in order on one stream
    pipelined = args.pipeline and not args.sequential

    def step(ev=None, pipe=pipelined):
        if ev is not None:
            ev[0].record(stream)
        if n:
            if pipe:
                v.verify_device_pipelined(d["R"].data_ptr(), d["S"].data_ptr(), d["K"].data_ptr(), d["M"].data_ptr(),
                                          ENVELOPE, ENVELOPE, n, d_local.data_ptr(), stream.cuda_stream,
                                          fin_stream.cuda_stream)
            else:
                v.verify_device(d["R"].data_ptr(), d["S"].data_ptr(), d["K"].data_ptr(), d["M"].data_ptr(), ENVELOPE,
                                ENVELOPE, n, d_local.data_ptr(), stream.cuda_stream)
        if ev is not None:
            ev[1].record(stream)
        if ws > 1:
            with torch.cuda.stream(fin_stream if pipe else stream):
                allgather_bitmap(d_local, ws, d_all)

    def check_round():
        words = round_bitmap(d_local, n_total, ws, d_all)
        got = bitmap_to_bool(words.cpu().numpy().view(np.uint64), n_total)
        assert (got == expect).all(), f"round bitmap differs from the expected bits at {np.nonzero(got != expect)[0][:8]}"

    # Settle: the table builds just ran the GPU flat out; keep launching rounds for --settle-s seconds so that
    # clocks and address-translation caches reach steady state before the W warmup + K timed steps.
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < args.settle_s:
        step()
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    check_round()

    # HIP events on the launch stream: pipelined, a pair around every step's comb kernel (its finish runs on
    # fin_stream); sequential, ONE pair around the whole timed region -- a pair per step adds two timestamp packets
    # between the launches (the finish -> next comb gap grew from ~11 to ~20 us, profiles/r04/shard/), so the
    # launch pair's average is the region's time / K (the ~11-us gap between launches included)
    # (N > 1: the region holds the all-gathers too; the kernels' own time is taken after it, untimed for `value`,
    # rather than by an event pair per step inside it -- two event records cost ~7.5 us per step on the GPU,
    # profiles/r05/shard/timing_events.txt, 4-5 % of an 8-GPU step)
    per_step = pipelined
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps if per_step else 1)]
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if not per_step:
        evs[0][0].record(stream)
    for k in range(args.steps):
        step(evs[k] if per_step else None)
    if not per_step:
        evs[0][1].record(stream)
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if per_step:
        kern_avg = float(np.mean([a.elapsed_time(b) for a, b in evs]))  # pipelined: the comb kernel
    else:
        kern_avg = evs[0][0].elapsed_time(evs[0][1]) / args.steps  # the comb + finish pair
    if ws > 1 and not per_step and n:
        kern_avg = time_device(v, stream, d, n, args.steps, torch)[0]  # this rank's launch pairs without the gathers
    if ws > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    check_round()  # the bitmap of the last timed step, assembled from every rank's shard

    # the same K rounds without pipelining (labelled figure): kernel, finish and all-gather of a round in order
    seq = None
    if pipelined and not args.no_extras:
        sev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        for _ in range(2):
            step(pipe=False)
        if ws > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0s = time.perf_counter()
        for k in range(args.steps):
            step(sev[k], pipe=False)
        torch.cuda.synchronize()
        if ws > 1:
            dist.barrier()
        sdt = time.perf_counter() - t0s
        if ws > 1:
            t = torch.tensor([sdt], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            sdt = float(t.item())
        check_round()
        seq = {"value": n_total * args.steps / sdt, "ms_per_step": sdt / args.steps * 1e3,
               "kernel_pair_avg_ms": float(np.mean([a.elapsed_time(b) for a, b in sev])),
               "note": "rounds not pipelined: comb, finish and all-gather of one round on one stream"}

    # weak-scaling figure (labelled, not the headline): every rank verifies the WHOLE round
    weak = None
    if not args.no_extras:
        dw = to_device(torch, dev, R, S, key_idx, msg) if ws > 1 else d
        wb = torch.zeros((n_total + 63) // 64, dtype=torch.int64, device=dev)
        dw["B"] = wb
        time_device(v, stream, dw, n_total, 2, torch)
        if ws > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.steps):
            v.verify_device(dw["R"].data_ptr(), dw["S"].data_ptr(), dw["K"].data_ptr(), dw["M"].data_ptr(),
                            ENVELOPE, ENVELOPE, n_total, wb.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        if ws > 1:
            dist.barrier()
        wdt = time.perf_counter() - t
        if ws > 1:
            tt = torch.tensor([wdt], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            wdt = float(tt.item())
        weak = {"value": n_total * ws * args.steps / wdt, "unit": "verifies/s", "scaling": "weak",
                "sigs_per_gpu": n_total, "ms_per_step": wdt / args.steps * 1e3,
                "note": "every rank verifies a whole 2^20 round (no exchange)"}
        if dw is not d:
            del dw
        got = bitmap_to_bool(wb.cpu().numpy().view(np.uint64), n_total)
        assert (got == expect).all()

    extras = {}
    if rank == 0 and not args.no_extras and ws == 1:
        # the per-GPU shard of an 8-GPU node (131,072 signatures): kernel time with the finish width it selects
        n8 = shard_bounds(n_total, 0, 8)[1]
        # (warm first: the shard's comb variant -- 8-wave blocks, paired priorities -- is not the 2^20 round's, and
        # its first launch loads the kernel, ~10 us on a 50-launch average; then the median of 5 samples)
        time_device(v, stream, d, n8, 5, torch)
        s8 = sorted(time_device(v, stream, d, n8, 50, torch) for _ in range(5))
        k8, w8 = s8[2]
        # the same shard pipelined over two streams (as bench runs at N = 8, minus the all-gather)
        torch.cuda.synchronize()
        tp = time.perf_counter()
        for _ in range(50):
            v.verify_device_pipelined(d["R"].data_ptr(), d["S"].data_ptr(), d["K"].data_ptr(), d["M"].data_ptr(),
                                      ENVELOPE, ENVELOPE, n8, d["B"].data_ptr(), stream.cuda_stream,
                                      fin_stream.cuda_stream)
        torch.cuda.synchronize()
        p8 = (time.perf_counter() - tp) * 1e3 / 50
        if args.replica_only:  # (no shard / latency legs before the replica legs)
            extras["replica_flush_2^20"] = replica_round_leg(v, seeds, pub, R, S, key_idx, msg, expect, rounds=20)
            print(json.dumps({"replica_only": extras["replica_flush_2^20"]}), flush=True)
            return
        extras["shard_of_8"] = {"sigs": n8, "kernel_ms": k8, "wall_ms_per_launch": w8,
                                "verifies_per_s_per_gpu": n8 / (k8 * 1e-3), "pipelined_wall_ms_per_launch": p8,
                                "kernel_ms_5_samples": [a for a, _ in s8], "pmc": shard_pmc(n8),
                                "note": "device-resident launches over the shard one GPU of 8 verifies"}
        # p50 latency of a 4096-signature round (config #5 batch size), device-resident
        lat = []
        n4 = min(4096, n)
        for it in range(args.latency_iters + 5):
            torch.cuda.synchronize()
            t = time.perf_counter()
            v.verify_device(d["R"].data_ptr(), d["S"].data_ptr(), d["K"].data_ptr(), d["M"].data_ptr(), ENVELOPE,
                            ENVELOPE, n4, d["B"].data_ptr(), stream.cuda_stream)
            torch.cuda.synchronize()
            if it >= 5:
                lat.append((time.perf_counter() - t) * 1e3)
        extras["p50_ms_4k_round"] = float(np.median(lat))
        extras["p99_ms_4k_round"] = float(np.percentile(lat, 99))
        # config #5: 2^24 sigs/s offered to an 8-GPU node = 2^21 per GPU; and back-to-back 4k batches
        # (>= 10k batches for the p50 / p99, as SURVEY §8d asks: 20 s at 512 batches/s)
        extras["stream_4k"] = {"offered_2^21_per_gpu": stream_latency(v, R, S, key_idx, msg, float(1 << 21),
                                                                      duration_s=args.stream_s),
                               "offered_2^21_per_gpu_pageable": stream_latency(v, R, S, key_idx, msg, float(1 << 21),
                                                                               duration_s=args.stream_s / 2,
                                                                               pinned=False),
                               "back_to_back": stream_latency(v, R, S, key_idx, msg, float("inf"))}
        # the replica legs (host-heavy) right after the config-#5 legs: after the e2e / votes / CPU legs the same leg
        # ran 3.6-3.9 ms against 3.1 ms in a fresh process on the same box (profiles/r06/final_a/, final_d/), and
        # with the replica legs BEFORE them the offered config-#5 leg saw one 17-40-ms GPU-side wait in each of
        # three lines (profiles/r06/final_b/ c/ e/: the host polling every ~20 us meanwhile), in none of three without
        extras["replica_flush_2^20"] = replica_round_leg(v, seeds, pub, R, S, key_idx, msg, expect, rounds=20)
        # the same round through pbft_replica_create_multi over this context + 1 clone (one slice each; on a node the
        # contexts would be two GPUs with a PCIe link each -- here both share this GPU and its link)
        extras["replica_flush_2^20_2ctx"] = replica_round_leg(v, seeds, pub, R, S, key_idx, msg, expect, rounds=20,
                                                                n_ctx=2)
        # the reference-shaped ingress: one message at a time on one thread
        extras["replica_ingress_2^20"] = replica_ingress_leg(v, seeds, pub, S, ~expect, n_seq)
        extras["e2e_2^20"] = e2e_host_round(v, R, S, key_idx, msg, expect, torch)
        extras["e2e_votes_2^20"] = e2e_votes_round(v, R, S, key_idx, msg, expect, torch)
        extras["votes_device_2^20"] = votes_device_round(v, d, msg, expect, stream, torch, dev)
        extras["config2"] = config2_leg(v, torch, dev, stream, cpu=not args.no_cpu)
        extras["config3"] = config3_leg(v, torch, dev, stream, cpu=not args.no_cpu)
        extras["shuffled_2^20"] = shuffled_leg(v, d, n, stream, torch, dev, expect)
        # the C ABI's single-process multi-GPU form on this process's one GPU (a 1-rank RCCL communicator): its
        # bitmap must equal the headline path's; unmeasured on 8 GPUs in this pipeline
        rate, ms_multi, got_multi = c_abi_multi_round([v], R, S, key_idx, msg, expect, torch, 10)
        head = bitmap_to_bool(round_bitmap(d_local, n_total, ws, d_all).cpu().numpy().view(np.uint64), n_total)
        assert (got_multi == head).all()
        extras["c_abi_multi_1gpu"] = {"value": rate, "unit": "verifies/s", "ms_per_step": ms_multi, "gpus": 1,
                                      "bitmap_equals_headline": True,
                                      "path": "pbft_multi_create + pbft_verify_batch_device_multi (1-rank RCCL "
                                              "communicator): shard verify + in-place ncclAllGather, C ABI only"}
        extras["set_keys_ms"] = set_keys_ms
        extras["set_keys_phases_ms"] = set_keys_phases
        extras.update(rekey_legs(v, pub, d, n, stream, torch, expect))
        extras["key_plans_2^20"] = plan_legs(v, pub, d, n, stream, torch)

    if rank == 0:
        total = n_total * args.steps
        value = total / dt
        # the dominant kernel: comb_kernel alone when pipelined (its launch is what the events bracket),
        # else the comb + finish pair
        ppv = products_comb(pb, pa) if pipelined else products_per_verify(pb, pa)
        products = ppv * n / (kern_avg * 1e-3)
        cpu = {} if args.no_cpu or ws > 1 else cpu_baselines(pub, R, S, key_idx, msg, expect)
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
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32 (GF(2^255-19) radix 2^25.5 limbs, 32x32->64 products)",
            "data": "synthetic: 256 replica keys, 85-B signed Prepare/Commit envelopes, GPU-signed (RFC 8032), "
                    "0.1% of signatures corrupted (bitmap checked)",
            "config": {"workload": "config#4: one round of n=256 replicas x 2048 seqs x {Prepare,Commit} = 2^20 "
                                   "signatures, sharded by index over the GPUs",
                       "sigs_per_step": n_total, "sigs_per_gpu": n, "msg_len": ENVELOPE, "settle_s": args.settle_s,
                       "parallelism": f"shard-by-index x{ws}" + (" + RCCL all-gather of bitmaps" if ws > 1 else "")},
            "roofline": {"bound": "valu", "achieved": products / 1e12, "peak": VALU_MAD_PEAK_PER_S / 1e12,
                         "unit": "T products/s (v_mad_u64_u32)", "frac": products / VALU_MAD_PEAK_PER_S,
                         "peak_source": "profiles/r03/valu_clock.txt: v_mad_u64_u32 issue, 4.53 cycles per "
                                        "wave-instruction per SIMD at the in-kernel clock 2.157 GHz",
                         "peak_at_2.4GHz": mad_peak_at(2.4e9) / 1e12,
                         "traffic": pmc.get("traffic_bytes_per_launch"),
                         "traffic_source": pmc.get("source"),
                         "valu_busy_pct": pmc.get("valu_busy_pct"),
                         "valu_insts_per_sig": pmc.get("valu_insts_per_sig"),
                         "valu_insts_per_sig_comb": pmc.get("valu_insts_per_sig_comb"),
                         "gather_bytes_algorithmic": (gather_bytes_per_verify(pb, pa) + INPUT_BYTES) * n,
                         "kernel": (f"comb_kernel<85, plan PA={pa}> (PB={pb}) over this rank's shard (HIP events on "
                                    f"its stream; the finish runs on the second stream)") if pipelined else
                                   f"comb_kernel<85, plan PA={pa}> (PB={pb}) + finish over this rank's shard",
                         "kernel_avg_ms": kern_avg, "products_per_verify": ppv},
            "pipelined": pipelined,
            "sequential_rounds": seq,
            "weak_scaling": weak,
            "cpu_baseline": cpu.get("port"),
            "cpu_baseline_openssl": cpu.get("openssl"),
            "vs_cpu_openssl": value / cpu["openssl"]["value"] if "openssl" in cpu else None,
        }
        line.update(extras)
        print(json.dumps(line), flush=True)
    v.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
