"""World-size-2 gloo test of the shard + bitmap all-gather path (no GPU)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT, golden_batches


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, expected, q):
    import torch.distributed as dist
    from pbft_amd.dist import allgather_bitmap, assemble, shard_bounds, shard_words
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = len(expected)
    lo, hi = shard_bounds(n, rank, world)
    # stand-in for this rank's GPU result: its shard of the oracle's expected bits
    bits = np.zeros(shard_words(n, world) * 64, dtype=np.uint8)
    bits[: hi - lo] = expected[lo:hi]
    local = torch.from_numpy(np.packbits(bits, bitorder="little").view(np.int64).copy())
    full = assemble(allgather_bitmap(local, world), n, world)
    if rank == 0:
        q.put(full.numpy().view(np.uint64).copy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_bitmap_allgather_gloo(golden, world):
    b = dict(golden_batches(golden))[85]
    exp = b["expected"].astype(np.uint8)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, exp, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = np.packbits(np.concatenate([exp, np.zeros((-len(exp)) % 64, np.uint8)]), bitorder="little").view(np.uint64)
    assert (got == want).all()


def test_shard_bounds_cover_and_align():
    from pbft_amd.dist import shard_bounds
    for n in (1, 63, 64, 65, 1000, 1 << 20, (1 << 20) + 7):
        for w in (1, 2, 3, 4, 8):
            seen = 0
            for r in range(w):
                lo, hi = shard_bounds(n, r, w)
                assert lo == seen and lo % 64 == 0 or lo == n
                seen = hi
            assert seen == n
