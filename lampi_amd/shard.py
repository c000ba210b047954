"""Multi-GPU sharding of fragment batches (one process per GPU, no data-path collective).

Fragments are independent, so a global batch of fragments k = 0..n-1 splits round-robin
over the ranks (rank r owns k = r (mod N), BASELINE.json config D) and every GPU checksums
its own shard from its own HBM.  The only cross-rank traffic is bookkeeping after the fact:
the max of the per-rank times and, for verification, the digests below (XOR of checksums;
sum of c_k * (2k+1) mod 2^32), which combine across shards with XOR and + respectively.
"""
from __future__ import annotations

import numpy as np

__all__ = ["shard_indices", "shard_count", "digest", "combine_digests", "allreduce_digest"]


def shard_count(n_global: int, rank: int, world: int) -> int:
    """Number of fragments k < n_global with k = rank (mod world)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return max(0, (n_global - rank + world - 1) // world)


def shard_indices(n_global: int, rank: int, world: int) -> np.ndarray:
    """Global fragment indices owned by `rank` (round-robin)."""
    return np.arange(rank, n_global, world, dtype=np.uint64)


def digest(vals: np.ndarray, k_index: np.ndarray) -> tuple[int, int]:
    """(XOR c_k, sum c_k*(2k+1) mod 2^32) over the given fragments."""
    v = np.asarray(vals, dtype=np.uint64)
    k = np.asarray(k_index, dtype=np.uint64)
    if v.size == 0:
        return 0, 0
    x = int(np.bitwise_xor.reduce(v))
    s = int(((v * (2 * k + 1)) & np.uint64(0xFFFFFFFF)).sum() & 0xFFFFFFFF)
    return x & 0xFFFFFFFF, s


def combine_digests(parts) -> tuple[int, int]:
    """Combine per-shard digests into the digest of the whole batch."""
    x, s = 0, 0
    for px, ps in parts:
        x ^= px
        s = (s + ps) & 0xFFFFFFFF
    return x, s


def allreduce_digest(local: tuple[int, int], group=None) -> tuple[int, int]:
    """Combine this rank's shard digest with every other rank's (torch.distributed).

    The per-rank digests are all-gathered and combined here: RCCL/NCCL have no bitwise-XOR
    reduction, so an all_reduce(BXOR) would only work on gloo."""
    import torch
    import torch.distributed as dist

    # RCCL: a tensor on this rank's own device (bench.py set it with torch.cuda.set_device)
    dev = "cpu" if dist.get_backend(group) == "gloo" else torch.device("cuda", torch.cuda.current_device())
    mine = torch.tensor([local[0], local[1]], dtype=torch.int64, device=dev)
    parts = [torch.empty_like(mine) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, mine, group=group)
    return combine_digests([(int(p[0].item()), int(p[1].item())) for p in parts])
