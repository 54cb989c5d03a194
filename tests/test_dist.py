"""Multi-rank (gloo, CPU) tests of the sharded round: shard layout, per-rank verification of the shard, the bitmap
all-gather and the assembly of the round's bitmap -- the same functions bench.py's multi-GPU step runs
(pbft_amd.dist.shard_bounds / round_bitmap), with the C oracle verifying each rank's shard in place of the GPU."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT, golden_batches


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_bits(b, lo, hi):
    o = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    vp = ctypes.c_void_p
    o.oracle_verify_batch.argtypes = [vp, ctypes.c_uint32, vp, vp, vp, vp, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint64, vp, ctypes.c_int]
    n = hi - lo
    out = np.zeros(max(n, 1), np.uint8)
    if n:
        R, S = np.ascontiguousarray(b["R"][lo:hi]), np.ascontiguousarray(b["S"][lo:hi])
        K, M = np.ascontiguousarray(b["key_idx"][lo:hi]), np.ascontiguousarray(b["msg"][lo:hi])
        assert o.oracle_verify_batch(b["keys"].ctypes.data, len(b["keys"]), R.ctypes.data, S.ctypes.data,
                                     K.ctypes.data, M.ctypes.data, 85, 85, n, out.ctypes.data, 1) == 0
    return out[:n]


def _worker(rank, world, port, n_total, q):
    import torch
    import torch.distributed as dist
    from conftest import golden_batches as gb
    from pbft_amd.dist import round_bitmap, shard_bounds, shard_words
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = dict(gb(np.load(os.path.join(ROOT, "tests", "golden", "verify_vectors.npz"))))[85]
    b = {k: v[:n_total] if k in ("R", "S", "key_idx", "msg") else v for k, v in b.items()}
    lo, hi = shard_bounds(n_total, rank, world)
    bits = np.zeros(shard_words(n_total, world) * 64, dtype=np.uint8)
    bits[: hi - lo] = _oracle_bits(b, lo, hi)              # this rank verifies its own shard
    local = torch.from_numpy(np.packbits(bits, bitorder="little").view(np.int64).copy())
    full = round_bitmap(local, n_total, world)
    if rank == 0:
        q.put(full.numpy().view(np.uint64).copy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total", [(2, 1456), (3, 1456), (4, 1001), (4, 65), (8, 200)])
def test_sharded_round_bitmap_gloo(golden, world, n_total):
    """Ragged shards (1456 over 3 ranks; 65 over 4 leaves ranks 2, 3 empty; 200 over 8 leaves 4 empty)."""
    b = dict(golden_batches(golden))[85]
    exp = b["expected"][:n_total].astype(np.uint8)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=180)
        assert p.exitcode == 0
    want = np.packbits(np.concatenate([exp, np.zeros((-len(exp)) % 64, np.uint8)]), bitorder="little").view(np.uint64)
    assert len(got) == len(want) and (got == want).all()


def test_shard_bounds_cover_and_align():
    from pbft_amd.dist import shard_bounds, shard_words
    for n in (1, 63, 64, 65, 1000, 1 << 20, (1 << 20) + 7):
        for w in (1, 2, 3, 4, 8):
            seen = 0
            for r in range(w):
                lo, hi = shard_bounds(n, r, w)
                assert lo == seen and lo % 64 == 0 or lo == n
                assert (hi - lo + 63) // 64 <= shard_words(n, w)
                seen = hi
            assert seen == n
    assert shard_bounds(1 << 20, 0, 8) == (0, 131072)                  # the per-GPU shard of config #4 on 8 GPUs
