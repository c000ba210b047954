"""CPU: bench.py's multi-rank launch (VERDICT r1 "next" #1), rehearsed without a GPU.

`python bench.py --gpus N --dry-run` starts N rank processes itself (no WORLD_SIZE in the
environment), they rendezvous over gloo on 127.0.0.1, take their round-robin shards k = r
(mod N) of config B's first 1024 fragments, gather per-rank rows and combine their digests --
the same code path a GPU run takes, with the kernel replaced by the reference's committed
values (tests/golden/config_b_head.json).  The combined digest is checked here against the
oracle, independently of that file.
"""
import json
import os
import subprocess
import sys
from types import SimpleNamespace

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=timeout)


def _json_line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("gpus", [1, 2, 4, 8])
@pytest.mark.parametrize("mode", ["crc", "sum"])
def test_dry_run_launches_n_ranks(gpus, mode, oracle):
    r = _run(["--gpus", str(gpus), "--dry-run", "--steps", "3", "--warmup", "1", "--mode", mode])
    assert r.returncode == 0, r.stderr
    d = _json_line(r.stdout)
    assert d["n_gpus"] == gpus and d["dry_run"] is True
    assert [e["rank"] for e in d["per_gpu"]] == list(range(gpus))
    assert all(e["parity_ok"] for e in d["per_gpu"])
    assert sum(e["bytes"] for e in d["per_gpu"]) == 1024 * 4096
    assert d["config"]["fragments_per_gpu"] == 1024 // gpus
    # the combined digest equals the oracle's digest of the whole 1024-fragment batch
    vals = oracle.uniform_batch(2, 0, 1024, 4096, 0 if mode == "crc" else 1)
    from oracle.oracle import digest

    want = digest(vals)
    assert (int(d["parity"]["xor"], 16), int(d["parity"]["wsum"], 16)) == want
    assert d["parity"]["ok"] is True and d["parity"]["all_ranks_ok"] is True
    assert d["aggregate"]["roofline_frac"] > 0
    # the roofline object: payload bytes per launch, and beside them the 4-byte results (messages; + the 16-byte
    # descriptors with --desc)
    rf = d["roofline"]
    n = d["config"]["fragments_per_gpu"]
    assert rf["algorithmic_bytes_per_launch"] == n * 4096
    assert rf["incl_metadata"]["bytes"] == n * (4096 + 4) and rf["incl_metadata"]["frac"] >= rf["frac"]


@pytest.mark.parametrize("mode", ["crc", "sum"])
def test_config_d_eight_rank_dry_run(mode):
    """Config D's own N = 8 plan (32M x 16 KiB, 4M fragments = 64 GiB per rank) through the launch, shard
    plan, row gather and digest combine of an 8-GPU run: each rank contributes its committed shard digest,
    the combined digest must be the whole batch's (CRC: BASELINE.md's F2A5DDAD / 3383EB2F) and every rank's
    CRC XOR BASELINE.md's per-GPU value."""
    r = _run(["--config", "D", "--gpus", "8", "--dry-run", "--steps", "2", "--warmup", "1", "--mode", mode],
             timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 8 and d["dry_run"] is True
    assert [e["rank"] for e in d["per_gpu"]] == list(range(8))
    assert all(e["bytes"] == 64 << 30 for e in d["per_gpu"])
    assert d["config"]["fragments_per_gpu"] == 4194304 and d["config"]["frag_bytes"] == 16384
    assert "mod 8" in d["config"]["sharding"]
    assert d["parity"]["ok"] is True and d["parity"]["all_ranks_ok"] is True
    if mode == "crc":
        assert (d["parity"]["xor"], d["parity"]["wsum"]) == ("f2a5ddad", "3383eb2f")
        assert "per-GPU shard XOR" in d["parity"]["check"]


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "1", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_rank_failure_fails_the_launch():
    # --dry-run covers only 1024 fragments: 4 ranks x 512 is refused by every rank -> nonzero exit
    r = _run(["--gpus", "4", "--dry-run", "--frags", "512"])
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_gpu_run_without_gpus_fails_loudly():
    # no GPU here: two ranks must refuse rather than silently run one (the 1-GPU-box case)
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"])
    assert r.returncode != 0
    assert "need 2 GPUs" in r.stderr


def _plan(**kw):
    sys.path.insert(0, ROOT)
    import bench

    a = SimpleNamespace(frags=4194304, frag_bytes=4096, seed=2, config="B", shard=None)
    a.__dict__.update(kw)
    return bench, a


def test_config_d_plan_and_cap():
    bench, a = _plan(config="D")
    with pytest.raises(SystemExit, match="exceeds"):
        bench.shard_plan(a, 1, 0)      # 512 GiB on one GPU
    with pytest.raises(SystemExit, match="exceeds"):
        bench.shard_plan(a, 2, 1)      # 256 GiB per rank
    n, L, seed, k0, kstep, ng = bench.shard_plan(a, 4, 3)
    assert (n, L, seed, k0, kstep, ng) == (8388608, 16384, 3, 3, 4, 33554432)
    n, L, seed, k0, kstep, ng = bench.shard_plan(a, 8, 5)
    assert (n * L, k0, kstep) == (64 << 30, 5, 8)
    bench, a = _plan(config="D", shard=7)
    assert bench.shard_plan(a, 1, 0) == (4194304, 16384, 3, 7, 8, 33554432)
    with pytest.raises(SystemExit):
        bench.shard_plan(a, 2, 0)      # --shard is a single-GPU mode
    bench, a = _plan(shard=1)
    with pytest.raises(SystemExit):
        bench.shard_plan(a, 1, 0)      # --shard without config D


def test_config_d_shard_digests_committed():
    """Every config D shard has a committed digest (both modes), consistent with BASELINE.md."""
    sys.path.insert(0, ROOT)
    import bench

    xs, ws = 0, 0
    for g in range(8):
        got = bench.shard_golden(3, 33554432, 16384, True, 8, g)
        assert got is not None and got[0] == bench.CONFIG_D_SHARD_XOR[g]
        xs ^= got[0]
        ws = (ws + got[1]) & 0xFFFFFFFF
        assert bench.shard_golden(3, 33554432, 16384, False, 8, g) is not None
    assert (xs, ws) == (0xF2A5DDAD, 0x3383EB2F)  # BASELINE.md config D total


def test_shard_indices_match_fill_layout():
    bench, a = _plan()
    for world in (1, 2, 8):
        parts = []
        for r in range(world):
            n, L, seed, k0, kstep, ng = bench.shard_plan(SimpleNamespace(**{**a.__dict__, "frags": 8}), world, r)
            parts.append(np.arange(n, dtype=np.uint64) * kstep + k0)
        assert np.array_equal(np.sort(np.concatenate(parts)), np.arange(8 * world, dtype=np.uint64))
