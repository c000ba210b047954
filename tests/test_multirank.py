"""CPU: the N > 1 path (round-robin shards, no data-path collective) with gloo, world size 2 and 4.

Each rank checksums its own shard (here with the oracle, standing in for its GPU) and only
bookkeeping crosses ranks: the digests combine to the single-rank digest of the whole batch,
exactly as bench.py's per-rank parity check and config D's per-GPU digests assume.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from lampi_amd import shard


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, L, seed, q):
    import torch.distributed as dist

    from oracle.oracle import Restatement

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ref = Restatement()
    ks = shard.shard_indices(n, rank, world)
    assert ks.size == shard.shard_count(n, rank, world)
    vals = np.array([ref.uniform_batch(seed, int(k), 1, L, 0)[0] for k in ks], dtype=np.uint32)
    local = shard.digest(vals, ks)
    total = shard.allreduce_digest(local)
    q.put((rank, local, total))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_digest_equals_whole(world, oracle):
    n, L, seed = 3001, 1024, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, L, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    whole = shard.digest(oracle.uniform_batch(seed, 0, n, L, 0), np.arange(n, dtype=np.uint64))
    for _, _, total in res:
        assert total == whole
    assert shard.combine_digests([r[1] for r in sorted(res)]) == whole


def test_shard_partition_is_exact():
    for n in (0, 1, 7, 64, 1001):
        for world in (1, 2, 3, 8):
            ks = np.concatenate([shard.shard_indices(n, r, world) for r in range(world)])
            assert np.array_equal(np.sort(ks), np.arange(n, dtype=np.uint64))
            assert sum(shard.shard_count(n, r, world) for r in range(world)) == n


def test_config_d_shard_digests_combine():
    # config D per-GPU CRC XORs (GPU g owns k = g mod 8) combine to the total
    per_gpu = [0x54862C49, 0x046DA633, 0x53ABB493, 0xEB1A2E44, 0xB9EACC67, 0x0BEC3926, 0x937B2402, 0x3B821C43]
    x, _ = shard.combine_digests([(v, 0) for v in per_gpu])
    assert x == 0xF2A5DDAD
