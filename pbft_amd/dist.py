"""Multi-GPU sharding of a round batch and the bitmap exchange.

Signatures are independent, so a round of N signatures is split into
contiguous, 64-aligned shards (bitmap words never straddle ranks), one process
per GPU verifies its shard, and the only collective is an all-gather of the
per-rank bitmap words (RCCL over xGMI with backend "nccl"; gloo on CPU tests).
"""
from __future__ import annotations


def shard_bounds(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """[lo, hi) of rank's shard: contiguous, lo a multiple of 64."""
    words = (n_total + 63) // 64
    per = (words + world - 1) // world
    lo = min(n_total, rank * per * 64)
    hi = min(n_total, (rank + 1) * per * 64)
    return lo, hi


def shard_words(n_total: int, world: int) -> int:
    """Bitmap words every rank contributes (the largest shard's, others padded)."""
    words = (n_total + 63) // 64
    return (words + world - 1) // world


def allgather_bitmap(local, world: int, out=None):
    """All-gather equal-length int64 word tensors -> one concatenated tensor.

    Uses all_gather_into_tensor (one RCCL call, no host round trip) when the
    backend supports it, else the list form (gloo)."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return local
    if out is None:
        out = torch.empty(local.numel() * world, dtype=local.dtype, device=local.device)
    if dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(out, local)
    else:
        parts = list(out.chunk(world))
        dist.all_gather(parts, local)
        if parts[0].data_ptr() != out.data_ptr():
            out.copy_(torch.cat(parts))
    return out


def assemble(gathered_words, n_total: int, world: int):
    """Drop each rank's padding words and return the round's bitmap words."""
    import torch
    per = shard_words(n_total, world)
    words = (n_total + 63) // 64
    chunks = []
    for r in range(world):
        lo, hi = shard_bounds(n_total, r, world)
        nw = (hi - lo + 63) // 64
        chunks.append(gathered_words[r * per: r * per + nw])
    return torch.cat(chunks)[:words]


def round_bitmap(local, n_total: int, world: int, gathered=None):
    """The round's bitmap words from every rank's shard words (bench.py's exchange step and its check):
    one all-gather of the equal-length padded shards, then the padding words dropped."""
    if world == 1:
        return local[: (n_total + 63) // 64]
    return assemble(allgather_bitmap(local, world, gathered), n_total, world)
