#!/usr/bin/env python3
"""bench.py -- device-resident fragment-CRC throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], per GPU): 4,194,304 fragments x 4 KiB = 16 GiB,
device-resident, CRC-32/MPEG-2 (LA-MPI uicrc) of every fragment.  A "step" is one
lampi_msg_csum launch over the whole batch.  The payload is the SURVEY.md 8(d) synthetic
stream (seed 2) generated on the device before timing.  With N GPUs each rank owns the
round-robin shard k = r (mod N) of a global batch of N x 4M fragments (weak scaling, no
collective on the data path; torch.distributed is used only for the barrier and the
max-over-ranks time).

Prints ONE JSON line (rank 0):
  value      = bytes checksummed by all ranks / max-over-ranks wall time of the K steps, GiB/s
  roofline   = dominant kernel's algorithmic bytes per launch (= 16 GiB payload) / its
               average launch duration from HIP events on the launch stream, vs 8.0 TB/s
  cpu_baseline = the reference's uicrc (oracle/_ref, compiled from /root/reference) or the
               clean-room port, on this host's cores (1 and the affinity mask), over BASELINE
               config A exactly (seed 1, 1M x 1 KiB), digest-checked
  parity     = digest of all ranks' results (global fragment indices) vs committed digests
               (tests/golden/bench_digests.json, made by the oracle in the build
               container).  Only the cpu_baseline leg imports oracle/.

Multi-GPU: under torchrun (WORLD_SIZE set) WORLD_SIZE must equal --gpus; `python bench.py
--gpus N` without a launcher starts the N rank processes itself (the parent never touches the
GPU).  Every rank's kernel average is gathered into `per_gpu` (GiB/s and roofline fraction per
GPU) and `aggregate` (all bytes / slowest kernel / N x 8 TB/s).  A node with fewer GPUs than
ranks fails loudly.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--frags F] [--frag-bytes L]
       python bench.py --config D --gpus N   # 32M x 16 KiB over N >= 4 GPUs (<= 200 GiB per rank)
       python bench.py --config D --shard g  # GPU g's full 64 GiB shard of the 8-GPU partition, 1 GPU
       python bench.py --gpus 2 --dry-run    # CPU rehearsal of the rank launch (gloo, no kernel)
       python bench.py --e2e        # host-memory path (config E), for DESIGN.md
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident fragment-CRC GiB/s (batched); % of HBM-read roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
GIB = float(1 << 30)

# BASELINE.md oracle digests (CRC XOR, CRC WSUM) of the uniform configs
GOLDEN = {
    (2, 4194304, 4096): (0x959621BB, 0xC38D8899),
    (1, 1048576, 1024): (0xFEB61101, 0x41FADF13),
    (3, 33554432, 16384): (0xF2A5DDAD, 0x3383EB2F),
}
# CRC XOR of GPU g's shard (k = g mod 8), 8 GPUs
CONFIG_D_SHARD_XOR = [0x54862C49, 0x046DA633, 0x53ABB493, 0xEB1A2E44, 0xB9EACC67, 0x0BEC3926, 0x937B2402, 0x3B821C43]


def golden_digest(seed: int, n_total: int, L: int, crc: bool):
    """Committed digest of fragments 0..n_total-1 (tests/golden/bench_digests.json)
    or None.  bench.py checks parity against committed data only: the oracle is imported
    solely by the cpu_baseline leg."""
    if crc and (seed, n_total, L) in GOLDEN:
        return GOLDEN[(seed, n_total, L)]
    try:
        with open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")) as f:
            entries = json.load(f)["entries"]
    except (OSError, ValueError, KeyError):
        return None
    m = "crc" if crc else "sum"
    for e in entries:
        if (e["seed"], e["n_total"], e["frag_bytes"], e["mode"], e.get("nshard", 1)) == (seed, n_total, L, m, 1):
            return e["xor"], e["wsum"]
    # the whole batch from a complete set of committed shard digests (config D: 8 shards)
    shards = {}
    for e in entries:
        if (e["seed"], e["n_total"], e["frag_bytes"], e["mode"]) == (seed, n_total, L, m) and "nshard" in e:
            shards.setdefault(e["nshard"], {})[e["shard"]] = (e["xor"], e["wsum"])
    for ns, parts in shards.items():
        if len(parts) == ns:
            x, w = 0, 0
            for px, pw in parts.values():
                x, w = x ^ px, (w + pw) & 0xFFFFFFFF
            return x, w
    return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU). Without WORLD_SIZE in the environment, bench.py starts N rank "
                         "processes itself; under torchrun WORLD_SIZE must equal N")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--frags", type=int, default=None, help="fragments per GPU (default: the config's)")
    ap.add_argument("--frag-bytes", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--mode", choices=["crc", "sum"], default="crc")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--config", choices=["B", "C", "D"], default="B",
                    help="B: 4M x 4 KiB per GPU, seed 2 (default, weak scaling); "
                         "C: mixed 64 B - 64 KiB Zipf sizes, >= 4 GiB, seed 5 (1 GPU, descriptor batch); "
                         "D: 32M x 16 KiB over N GPUs, seed 3 (BASELINE config D; per-rank shard <= 200 GiB)")
    ap.add_argument("--shard", type=int, default=None,
                    help="with --config D on one GPU: checksum GPU g's full shard of the 8-GPU partition "
                         "(4M x 16 KiB = 64 GiB, k = g mod 8) and check BASELINE.md's per-GPU digest")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the rank launch (gloo, no GPU): per-rank checksums come from "
                         "tests/golden/config_b_head.json instead of a kernel; nothing is measured")
    ap.add_argument("--e2e", action="store_true", help="host-memory end-to-end path (config E)")
    ap.add_argument("--latency", action="store_true", help="small-batch call latency (eager, synchronous, graph)")
    ap.add_argument("--bcopy", action="store_true",
                    help="fused copy + checksum batch (lampi_frag_bcopy_batch) on the config B shape")
    ap.add_argument("--recv", action="store_true",
                    help="batched receive step (lampi_copy_to_app_batch) on the config B shape in GM slots")
    ap.add_argument("--alternate", action="store_true",
                    help="with --recv: one stream alternating GM (65,456 B) and IB (1,976 B) receive batches, each "
                         "from its own descriptor array, beside each alone (learned shapes per array)")
    ap.add_argument("--rows-hint", type=int, default=0,
                    help="LAMPI_CSUM_ROWS_HINT(r) for the descriptor batches of --desc, --bcopy and --recv: the "
                         "fragments' 4 KiB rows (e.g. 16 for GM's 65,456-byte payloads); 0 = none")
    ap.add_argument("--desc", action="store_true",
                    help="run the batch through descriptors (lampi_frag_csum_batch, the general kernel) "
                         "instead of the contiguous-message entry point (diagnostic)")
    args = ap.parse_args()
    # rehearsal knobs (not for measurements): the bookkeeping backend, and ranks sharing GPUs so the
    # N-rank flow can be exercised on a smaller box (LAMPI_BENCH_SHARE_GPU=1: rank r on GPU r % ndev)
    args.backend = os.environ.get("LAMPI_BENCH_BACKEND", "nccl")
    args.share_gpu = os.environ.get("LAMPI_BENCH_SHARE_GPU") == "1"
    if args.backend not in ("nccl", "gloo"):
        ap.error("LAMPI_BENCH_BACKEND must be nccl or gloo")
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.frags is None:
        args.frags = (1024 // args.gpus) if args.dry_run else 4194304
    return args


MAX_SHARD_BYTES = 200 << 30  # per-rank payload cap: 288 GB of HBM less the allocator's and runtime's share


def launch_ranks(args) -> int:
    """`python bench.py --gpus N` (N > 1) without a launcher: start N rank processes of this
    script, one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1), the
    same environment torchrun gives them.  This parent never touches the GPU (it does not even
    import torch), so the children are ordinary processes, not re-execs of a GPU process.  If
    a rank fails, the others are stopped and the parent exits with the failing rank's code."""
    import signal
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    def forward(signum, _frame):  # a launcher stopped by a time limit takes its ranks with it
        for q in procs:
            if q.poll() is None:
                q.send_signal(signal.SIGTERM)
        sys.exit(128 + signum)

    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    rc = 0
    live = list(procs)
    while live:
        time.sleep(0.05)
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.send_signal(signal.SIGTERM)
    return rc


def dist_setup(args):
    """Rank, world size and local rank from the launcher's environment; the world size must be
    the --gpus the driver asked for, and a node must have a GPU for every local rank."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    import torch.distributed as dist

    if args.dry_run:
        if world > 1:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        return rank, world, local
    import torch

    ndev = torch.cuda.device_count()
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if not args.share_gpu and (ndev < local_world or local >= ndev):
        raise SystemExit(f"bench.py: {local_world} ranks on this node need {local_world} GPUs; "
                         f"{ndev} visible (rank {rank}, local rank {local})")
    if ndev == 0:
        raise SystemExit("bench.py: no GPU visible")
    dev = local % ndev if args.share_gpu else local
    torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":  # RCCL: bookkeeping only (barrier, max time, digests)
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
    return rank, world, local


def _coll_device(args):
    """Bookkeeping tensors: CPU for gloo, else this rank's own GPU (set by dist_setup)."""
    import torch

    if args.dry_run or args.backend != "nccl":
        return "cpu"
    return torch.device("cuda", torch.cuda.current_device())


def barrier(world):
    import torch.distributed as dist

    if world > 1:
        dist.barrier()


def max_over_ranks(x: float, world: int, args=None) -> float:
    import torch
    import torch.distributed as dist

    if world == 1:
        return x
    dev = _coll_device(args) if args else torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_rows(row, world: int, args) -> list:
    """Every rank's `row` (list of floats), in rank order (all_gather; rank 0 reports them)."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return [list(row)]
    t = torch.tensor(row, dtype=torch.float64, device=_coll_device(args))
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [p.cpu().tolist() for p in parts]


def cpu_baseline():
    """BASELINE config A exactly (BASELINE.md "CPU-baseline plan"): the reference's uicrc
    (oracle/_ref, compiled from /root/reference/src/util/MemFunctions.cc) -- or the clean-room
    port where that library was not built -- over seed 1, 1,048,576 x 1,024 B, on 1 core and on
    every core of this process's affinity mask; both results are checked against config A's
    digest (feb61101 / 41fadf13)."""
    import numpy as np

    from lampi_amd import shard
    from oracle.oracle import Reference, Restatement

    seed, n, L = 1, 1048576, 1024
    want = GOLDEN[(seed, n, L)]
    port = Restatement()
    kind, fn, src = "port", port.uicrc_addr(), "oracle/libcsum_ref.so (clean-room restatement)"
    try:
        ref = Reference()
        kind, fn, src = "reference", ref.uicrc_addr(), "oracle/_ref/libref_memfunctions.so (reference MemFunctions.cc)"
    except (FileNotFoundError, OSError):
        pass
    buf = port.stream(seed, 0, n * L)
    out1 = np.empty(n, dtype=np.uint32)
    t1, _ = port.time_crc_fn(fn, buf, n, L, 1, out=out1)
    mask = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None  # cgroup v2 CPU quota (the box's CPU share), in whole CPUs
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(q) // int(period))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    cores = min([mask] + [c for c in (quota, int(omp) if omp and omp.isdigit() else None) if c])
    outn = np.empty(n, dtype=np.uint32)
    tn, _ = port.time_crc_fn(fn, buf, n, L, cores, out=outn)
    ks = np.arange(n, dtype=np.uint64)
    d1, dn = shard.digest(out1, ks), shard.digest(outn, ks)
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": round(n * L / GIB / t1, 4), "unit": "GiB/s", "cores": 1, "kind": kind,
        "sample": f"BASELINE config A exactly: {n} x {L} B fragments of stream seed {seed} (1 GiB), "
                  f"uicrc init 0xFFFFFFFF, {src}; {t1:.2f} s on 1 core",
        "parity_ok": bool(d1 == want and dn == want),
        "digest": f"{d1[0]:08x}/{d1[1]:08x} (config A: {want[0]:08x}/{want[1]:08x})",
        "all_cores": {"value": round(n * L / GIB / tn, 3), "cores": cores, "seconds": round(tn, 3),
                      "threads": f"one per usable CPU: min(affinity mask {mask} of the host's {os.cpu_count()} CPUs, "
                                 f"cgroup quota {quota}, OMP_NUM_THREADS {omp})"},
        "cpu_model": model,
    }


def read_traffic(config_key: str):
    """HBM bytes per launch from a committed rocprofv3 PMC run (tools/pmc_traffic.py)."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(config_key)
        return None if e is None else e
    except (OSError, ValueError):
        return None


def shard_golden(seed: int, n_total: int, L: int, crc: bool, nshard: int, shard_id: int):
    """Committed digest (XOR, WSUM with global k) of shard k = shard_id (mod nshard), or None."""
    try:
        with open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")) as f:
            entries = json.load(f)["entries"]
    except (OSError, ValueError, KeyError):
        return None
    for e in entries:
        if (e["seed"], e["n_total"], e["frag_bytes"], e["mode"], e.get("nshard", 1), e.get("shard", 0)) == \
                (seed, n_total, L, "crc" if crc else "sum", nshard, shard_id):
            return e["xor"], e["wsum"]
    return None


def shard_plan(args, world: int, rank: int):
    """(fragments on this rank n, L, seed, first global index k0, index step, global count) for
    the uniform configs -- checked before any GPU is touched.  Config D is 32M x 16 KiB over
    the ranks (or, with --shard g, GPU g's shard of the 8-GPU partition on one GPU); no rank may
    hold more than MAX_SHARD_BYTES."""
    n, L, seed = args.frags, args.frag_bytes, args.seed
    k0, kstep, n_global = rank, world, n * world  # round-robin shard k = rank (mod world)
    if args.config == "D":
        L, seed = 16384, 3
        if args.shard is not None:
            if world != 1 or not 0 <= args.shard < 8:
                raise SystemExit("--shard g (0..7) runs one 8-GPU config D shard on a single GPU")
            n, n_global, k0, kstep = 33554432 // 8, 33554432, args.shard, 8
        else:
            if 33554432 % world:
                raise SystemExit("config D: 32M fragments do not split evenly over this many GPUs")
            n, n_global = 33554432 // world, 33554432
        if n * L > MAX_SHARD_BYTES:
            raise SystemExit(f"config D on {world} GPU(s): {n * L / GIB:.0f} GiB per rank exceeds the "
                             f"{MAX_SHARD_BYTES / GIB:.0f} GiB per-GPU cap (use >= 4 GPUs, or --shard g)")
    elif args.shard is not None:
        raise SystemExit("--shard is a config D option")
    if n * L > MAX_SHARD_BYTES:
        raise SystemExit(f"{n * L / GIB:.0f} GiB per rank exceeds the {MAX_SHARD_BYTES / GIB:.0f} GiB per-GPU cap")
    return n, L, seed, k0, kstep, n_global


def _read_schedule(crc: bool, desc: bool, n: int, L: int, rows_hint: int) -> str:
    """The read-only kernel the library's dispatch picks for a uniform batch of n x L-byte fragments (16-byte-aligned
    buffer; lampi_msg_csum, or lampi_frag_csum_batch with --desc once the census has seen the batch), as
    launch_crc_msg / launch_sum_msg / launch_crc_desc / launch_sum_desc choose it."""
    R = (L + 4095) // 4096
    pow2 = L & (L - 1) == 0
    if desc:
        if not crc and rows_hint <= 1 and pow2 and 64 <= L <= 1024 and n * L >= 256 * 4096:
            return (f"sum_row4k_desc_kernel<{L // 16}> (learned: equal fragments -- one short-lived workgroup per "
                    f"{4096 // L} fragments, each chunk read at its own descriptor's address)")
        if rows_hint <= 1 and pow2 and 64 <= L <= (2048 if crc else 1024) and n * L >= 256 * 4096:
            return (f"crc_regular_kernel<{'kSum, ' if not crc else ''}kSub = {L // 64}> (learned: the descriptors are one "
                    f"contiguous run -- packed rows from d[0].addr, {4096 // L} fragments per 4 KiB row, every "
                    "descriptor checked)")
        if rows_hint > 1:
            return ("crc_light_frag_copy_kernel<DescSource> (read-only, row groups + crc_light_group_join_kernel)"
                    if crc and rows_hint >= 8 else "crc_stream_kernel<RowSegSource%s> (16-row segments)"
                    % ("" if crc else ", kSum"))
        if crc:
            if L % 4096 == 0 and R <= 7 and n >= 4096:
                return ("crc_regular_kernel<kDesc> (learned: equal whole-row fragments, config B's schedule with "
                        "per-fragment addresses; crc_light_pair_leftover_kernel for off-shape ones)")
            if R >= 8:
                return "crc_light_frag_copy_kernel<DescSource> (learned: one wave per fragment, read-only)"
            if 1024 < L <= 2048 and L % 16:
                return "crc_light_pair_copy_kernel<DescSource> (learned: two fragments per wave)"
            return "crc_stream_kernel<DescSource> (piece streams)"
        if 2 <= R <= 8 and n >= 4096:
            return "sum_copy_wg_kernel<DescSource> (learned: one fragment per short-lived workgroup)"
        if R > 1:
            return "sum_copy_wg_kernel<GroupSource<DescSource>> + sum_group_join_kernel (learned row groups)"
        if L <= 1024:
            return "crc_stream_kernel<DescSource, kSum> (piece streams, 256 fragments per workgroup)"
        if L <= 2048:
            return "sum_copy_waves_kernel<DescSource> (learned: one fragment per wave)"
        return "sum_copy_wg_kernel<DescSource> (learned: two one-row fragments per workgroup)"
    if not crc and pow2 and 64 <= L <= 1024 and n * L >= 256 * 4096:
        return (f"sum_row4k_kernel<{L // 16}> (one short-lived 128-thread workgroup per 4 KiB of the message, "
                f"{4096 // L} fragments each)")
    if pow2 and 64 <= L <= (2048 if crc else 1024) and n * L >= 256 * 4096:
        return f"crc_regular_kernel<{'kSum, ' if not crc else ''}kSub = {L // 64}> (packed rows: {4096 // L} fragments per 4 KiB row)"
    if crc:
        if L % 4096 == 0 and R < 8 and L != 65536:
            return "crc_regular_kernel"
        if R >= 8:
            return "crc_light_frag_copy_kernel<MsgSource> (read-only, one wave per fragment; > 16 rows: 8-row groups)"
        if 1024 < L <= 2048 and L % 16 and n >= 256:
            return "crc_light_pair_copy_kernel<MsgSource> (two fragments per wave)"
        return "crc_stream_kernel<MsgSource> (piece streams)"
    if R > 1 and (n >= 256 or R > 8):
        return "sum_copy_wg_kernel<MsgSource> (one fragment per short-lived workgroup, or row groups)"
    if L <= 2048 and n >= 256:
        return "sum_copy_waves_kernel<MsgSource> (one fragment per wave)"
    if n >= 256:
        return "sum_copy_wg_kernel<MsgSource> (one fragment per short-lived workgroup)"
    return "crc_regular_kernel (kSum)" if L % 4096 == 0 else "crc_stream_kernel<MsgSource, kSum>"


def _copy_schedule(crc: bool, src: str, L: int, rows_hint: int) -> str:
    """The kernels a uniform batch of L-byte descriptor copies / receives runs once the stream's census
    has landed (frag_csum.hip learned_rows_hint: kShapeRows 8 CRC / kShapeRowsSum 4 SUM, pairs at <= 2 KiB)."""
    rows = max(1, -(-L // 4096))
    W = rows_hint if rows_hint > 1 else (rows if rows >= (8 if crc else 4) else 1)
    if crc:
        if rows_hint <= 1 and L <= 2048:
            return f"crc_light_pair_copy_kernel<{src}> (two fragments per wave) + crc_light_pair_leftover_kernel"
        return (f"crc_light_frag_copy_kernel<{src}>" +
                (f" ({W}-wave row groups + crc_light_group_join_kernel)" if W > 1 else ""))
    if W > 1:
        return f"sum_copy_wg_kernel<GroupSource<{src}>> ({W} row groups) + sum_group_join_kernel"
    if rows_hint <= 1 and L <= 2048:
        return f"sum_copy_waves_kernel<{src}> (one fragment per wave, four per workgroup)"
    return f"sum_copy_wg_kernel<{src}> (one 128-thread workgroup per fragment)"


def _recv_schedule(crc: bool, L: int, rows_hint: int) -> str:
    """The receive step's kernels: row groups zero the verdicts in their first launch, the other schedules
    after zero_verdicts_kernel (frag_csum.hip launch_copy_to_app)."""
    k = _copy_schedule(crc, "RecvSource", L, rows_hint)
    return k if "row groups" in k else "zero_verdicts_kernel + " + k


def _warm(fn, warmup: int, min_s: float = 0.5):
    """W untimed calls, then more until min_s has passed (as the config B / C warm-ups: the clocks of a fresh
    process ramp, and a copy shape dips for ~20 dispatches before it settles); returns the
    last call's result."""
    import torch

    t = time.perf_counter()
    res, i = None, 0
    while i < warmup or time.perf_counter() - t < min_s:
        res = fn()
        i += 1
        if i % 50 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return res


def _traffic(key: str, field: str = "hbm_bytes_per_launch"):
    """A field of a committed PMC traffic entry (profiles/traffic.json), or None."""
    e = read_traffic(key)
    return None if e is None else e.get(field)


def run_device(args):
    """One rank of the device-resident bench: fill this rank's shard in HBM, time K launches."""
    import numpy as np
    import torch

    from lampi_amd import shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    n, L, seed, k0, kstep, n_global = shard_plan(args, world, int(os.environ.get("RANK", "0")))
    rank, world, local = dist_setup(args)
    crc = args.mode == "crc"
    # global fragment indices (not needed by config D's dry run, whose shards are 4M fragments)
    ks = None if args.dry_run and args.config == "D" else np.arange(n, dtype=np.uint64) * np.uint64(kstep) + np.uint64(k0)

    if args.dry_run and args.config == "D":
        # CPU rehearsal of config D's N-GPU plan (32M x 16 KiB, 64 GiB per rank at N = 8): no kernel and
        # no per-fragment values; the rank's shard digest is the committed one (tests/golden/
        # bench_digests.json, the oracle's, whose CRC XORs are BASELINE.md's per-GPU values)
        shard_dig = shard_golden(seed, n_global, L, crc, world, rank)
        if shard_dig is None:
            raise SystemExit(f"--dry-run of config D needs committed {world}-shard digests (there are 8)")
        head, box = None, {}

        def run():
            box["vals"] = None
    elif args.dry_run:
        # CPU rehearsal: no kernel; the rank's "checksums" are the reference's, committed
        with open(os.path.join(ROOT, "tests", "golden", "config_b_head.json")) as f:
            head = json.load(f)
        if (seed, L) != (head["seed"], head["frag_bytes"]) or n_global > head["n"]:
            raise SystemExit(f"--dry-run covers config B's first {head['n']} fragments (seed 2, 4 KiB)")
        table = np.array(head["crc" if crc else "sum"], dtype=np.uint32)
        box = {}

        def run():
            box["vals"] = table[ks.astype(np.int64)]
    else:
        from lampi_amd import device as dv

        mode = dv.CRC32 if crc else dv.SUM32
        stream = torch.cuda.current_stream()
        buf = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        dv.fill_stream_frags(buf, n, L, seed, k0=k0, kstep=kstep)
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        if args.desc:
            descs = dv.make_descs(buf, np.arange(n, dtype=np.uint64) * L, np.full(n, L, np.uint64))
            run = lambda: dv.frag_csum_batch(descs, mode=mode, out=out, rows_hint=args.rows_hint)  # noqa: E731
        else:
            run = lambda: dv.msg_csum(buf, L, mode=mode, out=out)  # noqa: E731
        torch.cuda.synchronize()

    def sync():
        if not args.dry_run:
            torch.cuda.synchronize()

    # warm-up: the W launches, then more until 0.5 s have passed (the first dispatches of a fresh
    # process ramp from 2.8-3.4 ms down to the steady 2.63 ms: clock/power ramp)
    nw, t_w = 0, time.perf_counter()
    while nw < args.warmup or (not args.dry_run and time.perf_counter() - t_w < 0.5):
        run()
        sync()
        nw += 1

    barrier(world)
    sync()
    if args.dry_run:
        t0 = time.perf_counter()
        kern_ms = []
        for i in range(args.steps):
            ts = time.perf_counter()
            run()
            kern_ms.append((time.perf_counter() - ts) * 1e3)
    else:
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        t0 = time.perf_counter()
        evs[0].record(stream)
        for i in range(args.steps):
            run()
            evs[i + 1].record(stream)
        torch.cuda.synchronize()
    barrier(world)
    t1 = time.perf_counter()
    wall = max_over_ranks(t1 - t0, world, args)
    if args.dry_run:
        vals = box["vals"]
    else:
        kern_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]
        vals = dv.as_u32(out)
    kern_avg_s = sum(kern_ms) / len(kern_ms) / 1e3

    # parity: this rank's shard digest (global fragment indices), combined over the ranks, vs
    # committed digests
    local = shard.digest(vals, ks) if vals is not None else tuple(shard_dig)
    if args.dry_run and args.config == "D":
        whole = shard.allreduce_digest(local) if world > 1 else local
        want = golden_digest(seed, n_global, L, crc)
        check = "dry run: committed per-shard digests combined over the ranks vs the whole-batch digest"
    elif args.dry_run:
        whole = shard.allreduce_digest(local) if world > 1 else local
        want = tuple(head["digest_crc" if crc else "digest_sum"]) if n_global == head["n"] else None
        check = "combined shard digests vs tests/golden/config_b_head.json (reference values)"
    elif args.shard is not None:
        whole = local
        want = shard_golden(seed, n_global, L, crc, 8, args.shard)
        check = f"config D shard {args.shard} of 8 (64 GiB): digest vs tests/golden/bench_digests.json" + \
                (" and BASELINE.md per-GPU XOR" if crc else "")
        if want is not None and crc and want[0] != CONFIG_D_SHARD_XOR[args.shard]:
            raise SystemExit("tests/golden/bench_digests.json disagrees with BASELINE.md")
    else:
        whole = shard.allreduce_digest(local) if world > 1 else local
        want = golden_digest(seed, n_global, L, crc)
        check = "full digest vs BASELINE.md / tests/golden/bench_digests.json"
    if want is not None:
        ok = whole == tuple(want)
        if args.config == "D" and world == 8 and crc:
            ok = ok and local[0] == CONFIG_D_SHARD_XOR[rank]
            check += " (per-GPU shard XOR too)"
        parity = {"check": check, "xor": f"{whole[0]:08x}", "wsum": f"{whole[1]:08x}", "ok": ok}
    else:
        parity = {"check": "no committed digest for this shape (tests/golden/make_bench_digests.py)",
                  "xor": f"{whole[0]:08x}", "wsum": f"{whole[1]:08x}", "ok": None}
    bad = 0 if parity["ok"] is not False else 1
    # per-rank rows: [kernel avg s, bytes, parity failure, local wall s]
    rows = gather_rows([kern_avg_s, float(n) * L, float(bad), t1 - t0], world, args)

    result = None
    if rank == 0:
        bytes_total = sum(r[1] for r in rows)
        value = bytes_total / GIB / wall * args.steps
        achieved = n * L / kern_avg_s / 1e9
        kmax = max(r[0] for r in rows)
        per_gpu = [{"rank": i, "bytes": int(r[1]), "kernel_avg_ms": round(r[0] * 1e3, 4),
                    "GiB_per_s": round(r[1] / GIB / r[0], 2),
                    "roofline_frac": round(r[1] / r[0] / 1e9 / HBM_PEAK_GBS, 4),
                    "parity_ok": r[2] == 0} for i, r in enumerate(rows)]
        # PMC traffic is recorded per kernel: the descriptor runs have no entry of their own
        cfg_key = f"{'crc' if crc else 'sum'}_{'desc_' if args.desc else ''}{n}x{L}"
        traffic = None if args.dry_run else read_traffic(cfg_key)
        kernel = "none (dry run)" if args.dry_run else _read_schedule(crc, args.desc, n, L, args.rows_hint)
        workload = (f"config D shard {args.shard} of 8: {n} x {L} B fragments k = {args.shard} (mod 8), seed 3"
                    if args.shard is not None else
                    f"{n} x {L} B fragments per GPU, device-resident, "
                    f"{'CRC-32/MPEG-2 (uicrc)' if crc else 'uicsum'}, "
                    f"{('one descriptor per fragment, LAMPI_CSUM_ROWS_HINT(%d)' % args.rows_hint) if args.desc and args.rows_hint > 1 else 'one descriptor per fragment (the schedule of the learned batch shape: roofline.kernel)' if args.desc else 'one contiguous message (roofline.kernel)'}")
        result = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_launches": nw,
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": (f"synthetic: splitmix64 stream seed {seed} (SURVEY.md 8(d)), generated on device"
                     if not args.dry_run else "dry run: committed config D shard digests" if args.config == "D"
                     else "dry run: reference checksums of config B's first fragments"),
            "config": {
                "workload": workload,
                "fragments_per_gpu": n, "frag_bytes": L, "bytes_per_gpu": n * L,
                **({"rows_hint": args.rows_hint} if args.desc and args.rows_hint else {}),
                "sharding": f"round-robin k = {'g' if args.shard is not None else 'rank'} (mod {kstep}), "
                            f"no collective",
            },
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None if traffic is None else traffic.get("hbm_bytes_per_launch"),
                "kernel": kernel,
                "kernel_avg_ms": round(kern_avg_s * 1e3, 4),
                "kernel_ms_min_median_max": [round(x, 4) for x in (min(kern_ms), sorted(kern_ms)[len(kern_ms) // 2], max(kern_ms))],
                "algorithmic_bytes_per_launch": n * L,
                # + the 16-byte descriptor read (--desc) and the 4-byte result write per fragment
                "incl_metadata": {"bytes": n * (L + (16 if args.desc else 0) + 4),
                                  "achieved": round(n * (L + (16 if args.desc else 0) + 4) / kern_avg_s / 1e9, 1),
                                  "frac": round(n * (L + (16 if args.desc else 0) + 4) / kern_avg_s / 1e9
                                                / HBM_PEAK_GBS, 4)},
                "traffic_source": None if traffic is None else traffic.get("source"),
                "sq_per_4KiB_row": None if traffic is None else traffic.get("sq_per_4KiB_row"),
                "note": "rank 0's kernel; every rank's in per_gpu",
            },
            "per_gpu": per_gpu,
            "aggregate": {"GiB_per_s_kernel": round(bytes_total / GIB / kmax, 2),
                          "roofline_frac": round(bytes_total / kmax / 1e9 / (HBM_PEAK_GBS * world), 4),
                          "note": "sum of all ranks' bytes / slowest rank's kernel average / (N x 8 TB/s)"},
            "parity": {**parity, "all_ranks_ok": all(r[2] == 0 for r in rows)},
        }
        if args.dry_run:
            result["dry_run"] = True
        if args.share_gpu and world > 1:
            result["rehearsal"] = (f"{world} ranks shared the visible GPU(s) (LAMPI_BENCH_SHARE_GPU=1, backend "
                                   f"{args.backend}): checks the N-rank flow; the numbers are not a scaling result")
        if world == 1 and not args.no_cpu_baseline and not args.dry_run and args.shard is None:
            result["cpu_baseline"] = cpu_baseline()
        else:
            result["cpu_baseline"] = None
    return rank, world, result


def run_mixed(args):
    """Config C: one descriptor batch of Zipf-sized fragments packed back to back (seed 5)."""
    import numpy as np
    import torch

    from lampi_amd import device as dv
    from lampi_amd import shard
    from lampi_amd.workload import zipf_lengths

    rank, world, _ = dist_setup(args)
    if world != 1:
        raise SystemExit("config C is a single-GPU configuration")
    lens = zipf_lengths(4 << 30)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.sum(dtype=np.uint64))
    buf = torch.empty(total, dtype=torch.uint8, device="cuda")
    dv.fill_stream(buf, seed=5)
    descs = dv.make_descs(buf, offs, lens)
    out = torch.empty(lens.size, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    mode = dv.CRC32 if args.mode == "crc" else dv.SUM32
    # warm-up: the W launches, then more until 0.3 s have passed -- a config C launch is ~0.75 ms and
    # the clocks of a fresh process ramp for ~100 launches (measured: 65.8 -> 70.8 -> 72.9% over the
    # first three batches of ten)
    t_w = time.perf_counter()
    nw = 0
    while nw < args.warmup or time.perf_counter() - t_w < 0.3:
        dv.frag_csum_batch(descs, mode=mode, out=out)
        nw += 1
        if nw % 50 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record(stream)
    for i in range(args.steps):
        dv.frag_csum_batch(descs, mode=mode, out=out)
        evs[i + 1].record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]
    kern_avg_s = sum(kern_ms) / len(kern_ms) / 1e3
    with open(os.path.join(ROOT, "tests", "golden", "fixtures.json")) as f:
        gold = json.load(f)["digests"]["C"]
    vals = dv.as_u32(out)
    got = shard.digest(vals, np.arange(lens.size, dtype=np.uint64))
    if mode == dv.CRC32:
        want = (gold["crc_xor"], gold["crc_wsum"])
    else:  # SUM: total of the sums and the weighted sum
        got = (int(np.sum(vals, dtype=np.uint64) & 0xFFFFFFFF), got[1])
        want = (gold["sum_total"], gold["sum_wsum"])
    # the north_star's one-wavefront-per-fragment schedule on the same batch, beside the product
    pw_out = torch.empty_like(out)
    for _ in range(args.warmup):
        dv.diag_frag_csum_batch_per_wave(descs, mode=mode, out=pw_out)
    torch.cuda.synchronize()
    pev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    pev[0].record(stream)
    for i in range(args.steps):
        dv.diag_frag_csum_batch_per_wave(descs, mode=mode, out=pw_out)
        pev[i + 1].record(stream)
    torch.cuda.synchronize()
    pw_s = sum(pev[i].elapsed_time(pev[i + 1]) for i in range(args.steps)) / args.steps / 1e3
    pw_same = bool(torch.equal(pw_out, out))
    achieved = total / kern_avg_s / 1e9
    meta = total + 20 * lens.size  # + the 16-byte descriptor read and the 4-byte result write
    traffic = read_traffic("crc_configC" if mode == dv.CRC32 else "sum_configC")
    print(json.dumps({
        "metric": METRIC, "value": round(total / GIB / (wall / args.steps), 2), "unit": "GiB/s", "n_gpus": 1,
        "steps": args.steps, "warmup": nw, "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: splitmix64 stream seed 5, Zipf(1.1) lengths 64 B..64 KiB (SURVEY.md 8(d))",
        "config": {"workload": f"config C: {lens.size} mixed fragments, {total} B, one descriptor batch "
                               "(lampi_frag_csum_batch)", "fragments": int(lens.size), "bytes": total},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": None if traffic is None else traffic["hbm_bytes_per_launch"],
                     "traffic_source": None if traffic is None else traffic.get("source"),
                     "sq_per_4KiB_row": None if traffic is None else traffic.get("sq_per_4KiB_row"),
                     "kernel": "crc_stream_kernel" if mode == dv.CRC32 else "crc_stream_kernel<kSum>",
                     "incl_metadata": {"bytes": meta, "achieved": round(meta / kern_avg_s / 1e9, 1),
                                       "frac": round(meta / kern_avg_s / 1e9 / HBM_PEAK_GBS, 4)},
                     "kernel_avg_ms": round(kern_avg_s * 1e3, 4),
                     "kernel_ms_min_median_max": [round(x, 4) for x in (min(kern_ms), sorted(kern_ms)[len(kern_ms) // 2],
                                                                          max(kern_ms))],
                     "algorithmic_bytes_per_launch": total},
        "one_wavefront_per_fragment": {"kernel": "crc_rows_kernel<DescSource>" if mode == dv.CRC32 else
                                       "sum_rows_kernel<DescSource>",
                                       "entry_point": "lampi_diag_frag_csum_batch_per_wave (internal diagnostic, "
                                                      "retired from the C ABI in round 5)",
                                       "kernel_avg_ms": round(pw_s * 1e3, 4),
                                       "frac": round(total / pw_s / 1e9 / HBM_PEAK_GBS, 4),
                                       "same_checksums": pw_same},
        "parity": {"check": f"full digest vs tests/golden/fixtures.json (config C, {args.mode})",
                   ("xor" if mode == dv.CRC32 else "sum"): f"{got[0]:08x}", "wsum": f"{got[1]:08x}",
                   "ok": got == want and pw_same},
        "cpu_baseline": None}))


def run_e2e(args):
    """Config E: a 256 MiB message in host memory through the library's host-message path
    (lampi_host_msg_csum / lampi_host_msg_bcopy, one C-ABI call per message: chunked H2D ||
    checksum kernels || D2H inside the library).  Reported beside the raw pinned H2D / D2H rates of
    the same box; every result is checked against the committed config E digests (and the copies
    against the message)."""
    import numpy as np
    import torch

    from lampi_amd import _lib, shard
    from lampi_amd._lib import check, lib as _clib

    torch.cuda.set_device(0)
    c = _clib()
    msg_bytes = 256 << 20
    with open(os.path.join(ROOT, "tests", "golden", "fixtures.json")) as f:
        gold = json.load(f)["digests"]["E"]
    from lampi_amd import device as dv

    pinned = torch.empty(msg_bytes, dtype=torch.uint8).pin_memory()
    staged = torch.empty(msg_bytes, dtype=torch.uint8, device="cuda")
    dv.fill_stream(staged, seed=gold["seed"])  # the message, generated on the device, then parked in host memory
    pinned.copy_(staged)
    torch.cuda.synchronize()
    pageable = pinned.numpy().copy()
    reps = max(3, min(args.steps, 10))

    def timed(fn):
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        return (time.perf_counter() - t0) / reps

    # raw PCIe rates of this box: pinned H2D and D2H of the whole message (torch copies).  The two-way
    # paths (bcopy, receive) are reported against min(H2D, D2H): a concurrent H2D || D2H pair of torch
    # copies on two streams measured 26.6 GiB/s per direction, below what the library's own pipeline
    # moves both ways (37-40), so it is no ceiling
    t_h2d = timed(lambda: (staged.copy_(pinned, non_blocking=True), torch.cuda.synchronize()))
    t_d2h = timed(lambda: (pinned.copy_(staged, non_blocking=True), torch.cuda.synchronize()))
    del staged
    h2d, d2h = msg_bytes / GIB / t_h2d, msg_bytes / GIB / t_d2h
    res = {}
    ok_all = True
    for L in (4096, 16384, 65456):
        nfr = (msg_bytes + L - 1) // L
        g = gold[str(L)]
        out = np.empty(nfr, dtype=np.uint32)
        ks = np.arange(nfr, dtype=np.uint64)
        row = {"fragments": int(nfr)}
        for src_kind, src_ptr in (("pinned", pinned.data_ptr()), ("pageable", pageable.ctypes.data)):
            out.fill(0)
            t = timed(lambda: check(c.lampi_host_msg_csum(src_ptr, msg_bytes, L, 0, nfr, 0xFFFFFFFF,
                                                          out.ctypes.data, 0), "lampi_host_msg_csum"))
            ok = nfr == g["n"] and shard.digest(out, ks) == (g["crc_xor"], g["crc_wsum"])
            ok_all &= ok
            row[f"csum_{src_kind}_src"] = {"GiB_per_s": round(msg_bytes / GIB / t, 2), "ms": round(t * 1e3, 3),
                                           "frac_of_pinned_h2d": round(msg_bytes / GIB / t / h2d, 4),
                                           "bit_exact": bool(ok)}
        # fused copy into NIC buffers: each payload behind a 72-byte header, buffers of L + 80 bytes
        # (65,456-byte payloads: GM's 64 KiB buffers, src/path/gm/state.h:48-57)
        stride = L + 80
        ring = torch.empty(nfr * stride, dtype=torch.uint8).pin_memory()
        ring_pg = np.empty(nfr * stride, dtype=np.uint8)
        for ring_kind, ring_arr, ring_ptr in (("pinned", ring.numpy(), ring.data_ptr() + 72),
                                              ("pageable", ring_pg, ring_pg.ctypes.data + 72)):
            out.fill(0)
            t = timed(lambda: check(c.lampi_host_msg_bcopy(pinned.data_ptr(), msg_bytes, L, 0, nfr, ring_ptr, stride,
                                                           0xFFFFFFFF, out.ctypes.data, 0), "lampi_host_msg_bcopy"))
            full = msg_bytes // L
            msg = pageable
            copy_ok = bool(np.array_equal(np.lib.stride_tricks.as_strided(ring_arr[72:], (full, L), (stride, 1)),
                                          msg[:full * L].reshape(full, L)))
            tail = msg_bytes - full * L
            if tail:
                copy_ok &= bool(np.array_equal(ring_arr[72 + full * stride:72 + full * stride + tail], msg[full * L:]))
            ok = nfr == g["n"] and shard.digest(out, ks) == (g["crc_xor"], g["crc_wsum"]) and copy_ok
            ok_all &= ok
            row[f"bcopy_pinned_src_{ring_kind}_ring"] = {
                "GiB_per_s": round(msg_bytes / GIB / t, 2), "ms": round(t * 1e3, 3),
                "frac_of_min_h2d_d2h": round(msg_bytes / GIB / t / min(h2d, d2h), 4),
                "slot_stride": stride, "bit_exact_and_copied": bool(ok)}
        # the receive side: the fragments now sit in the pinned ring (payload at +72 of each slot, its CRC
        # from the send call as the header's dataChecksum); one lampi_host_copy_to_app_batch call delivers
        # them all into an application buffer (ring order: one D2H per chunk) and verifies every checksum
        lens = np.full(nfr, L, dtype=np.uint32)
        lens[-1] = msg_bytes - (nfr - 1) * L
        frags = (_lib.HostRecvFrag * nfr)()
        fr = np.ctypeslib.as_array(ctypes.cast(frags, ctypes.POINTER(ctypes.c_uint8)), shape=(nfr * 32,)).view(
            np.dtype([("frag_off", "<u8"), ("app", "<u8"), ("app_len", "<i8"), ("length", "<u4"),
                      ("expected", "<u4")]))
        fr["frag_off"] = 72 + np.arange(nfr, dtype=np.uint64) * stride
        fr["app_len"] = lens
        fr["length"] = lens
        fr["expected"] = out
        copied = np.empty(nfr, np.int64)
        csums = np.empty(nfr, np.uint32)
        mask = np.empty((nfr + 31) // 32, np.uint32)
        nbad = ctypes.c_uint32(0)
        app_pin = torch.empty(msg_bytes, dtype=torch.uint8).pin_memory()
        app_pg = np.empty(msg_bytes, dtype=np.uint8)
        ring_pg[:] = ring.numpy()
        for ring_kind, ring_base, app_kind, app_arr, app_ptr in (
                ("pinned", ring.data_ptr(), "pinned", app_pin.numpy(), app_pin.data_ptr()),
                ("pinned", ring.data_ptr(), "pageable", app_pg, app_pg.ctypes.data),
                ("pageable", ring_pg.ctypes.data, "pageable", app_pg, app_pg.ctypes.data)):
            fr["app"] = app_ptr + np.arange(nfr, dtype=np.uint64) * L
            app_arr.fill(0)
            t = timed(lambda: check(c.lampi_host_copy_to_app_batch(ring_base, nfr * stride, ctypes.addressof(frags), nfr,
                                                                   copied.ctypes.data, csums.ctypes.data,
                                                                   mask.ctypes.data, ctypes.byref(nbad), 0),
                                    "lampi_host_copy_to_app_batch"))
            ok = (nbad.value == 0 and np.array_equal(copied, lens.astype(np.int64)) and np.array_equal(csums, out)
                  and not mask.any() and shard.digest(csums, ks) == (g["crc_xor"], g["crc_wsum"])
                  and np.array_equal(app_arr, pageable))
            ok_all &= ok
            row[f"recv_{ring_kind}_ring_{app_kind}_app"] = {
                "GiB_per_s": round(msg_bytes / GIB / t, 2), "ms": round(t * 1e3, 3),
                "frac_of_min_h2d_d2h": round(msg_bytes / GIB / t / min(h2d, d2h), 4),
                "bit_exact_and_delivered": bool(ok)}
        # the receiver's header check over the same ring (72-byte headers, GM residue; the headers hold no
        # stamped checksum here, so every one is reported -- this leg is timed, not checked)
        offs = np.arange(nfr, dtype=np.uint64) * stride
        t = timed(lambda: check(c.lampi_host_header_check_batch(ring.data_ptr(), nfr * stride, offs.ctypes.data, nfr,
                                                                72, 18, 68, mask.ctypes.data, ctypes.byref(nbad), 0),
                                "lampi_host_header_check_batch"))
        row["header_check_pinned_ring"] = {"headers_per_s": round(nfr / t), "ms": round(t * 1e3, 3),
                                           "nbad": int(nbad.value)}
        del ring, app_pin
        res[str(L)] = row
    print(json.dumps({"metric": "end-to-end host-memory fragment-CRC (config E: 256 MiB message in host memory, "
                                "one lampi_host_msg_csum / lampi_host_msg_bcopy call per message; the receive "
                                "side one lampi_host_copy_to_app_batch call per message)",
                      "unit": "GiB/s", "results": res, "pinned_h2d_GiB_per_s": round(h2d, 2),
                      "pinned_d2h_GiB_per_s": round(d2h, 2),
                      "reps": reps, "parity_ok": bool(ok_all)}), flush=True)


def run_bcopy(args):
    """copy n fragments into a staging array with the checksum fused
    (bcopy_uicrc / bcopy_uicsum of every fragment).  Roofline bytes = L read + L written.
    Timed: lampi_msg_bcopy (the value), the same work as a descriptor batch
    (lampi_frag_bcopy_batch) and torch's own device copy of the bytes (copy reference)."""
    import numpy as np
    import torch

    from lampi_amd import device as dv
    from lampi_amd import shard

    rank, world, _ = dist_setup(args)
    if world != 1:
        raise SystemExit("--bcopy is a single-GPU measurement")
    n, L = args.frags, args.frag_bytes
    mode = dv.CRC32 if args.mode == "crc" else dv.SUM32
    src = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    dv.fill_stream_frags(src, n, L, args.seed)
    dst = torch.zeros(n * L, dtype=torch.uint8, device="cuda")
    offs = np.arange(n, dtype=np.uint64) * L
    descs = dv.make_copy_descs(src, offs, dst, offs, np.full(n, L), np.full(n, L))
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()

    def timed(fn):
        _warm(fn, args.warmup)
        # (events at the ends of the K back-to-back calls: an event between two calls is a stream packet of
        # its own, ~6 us, which no application sends)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(args.steps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        return wall, e0.elapsed_time(e1) / args.steps / 1e3

    def check(tag):
        vals = dv.as_u32(out)
        copy_ok = bool(torch.equal(src, dst))
        want = golden_digest(args.seed, n, L, mode == dv.CRC32)
        got = shard.digest(vals, np.arange(n, dtype=np.uint64))
        if want is None:
            return {"check": f"{tag}: copy == source (no committed digest for this shape)", "xor": f"{got[0]:08x}",
                    "ok": copy_ok}
        return {"check": f"{tag}: full digest vs committed digest + copy == source", "xor": f"{got[0]:08x}",
                "ok": got == tuple(want) and copy_ok}

    wall, kern = timed(lambda: dv.msg_bcopy(src, L, dst, L, mode=mode, out=out))
    parity = check("msg_bcopy")
    dst.zero_()
    _, kern_desc = timed(lambda: dv.frag_bcopy_batch(descs, mode=mode, out=out, rows_hint=args.rows_hint))
    parity_desc = check("frag_bcopy_batch")
    # the GM receive shape: payloads 8 bytes past a 16-byte boundary (after a 72-byte header),
    # destinations aligned -- n-1 fragments of src[8 + k*L, ...)
    descs8 = dv.make_copy_descs(src, offs[:-1] + np.uint64(8), dst, offs[:-1], np.full(n - 1, L), np.full(n - 1, L))
    _, kern_desc8 = timed(lambda: dv.frag_bcopy_batch(descs8, n=n - 1, mode=mode, out=out, rows_hint=args.rows_hint))
    copy8_ok = bool(torch.equal(src[8:8 + (n - 1) * L], dst[:(n - 1) * L]))
    # the GM send shape: payloads gathered into ring slots right after the 72-byte header --
    # destinations 8 bytes past a 16-byte boundary, sources aligned
    descs_d8 = dv.make_copy_descs(src, offs[:-1], dst, offs[:-1] + np.uint64(8), np.full(n - 1, L), np.full(n - 1, L))
    _, kern_dst8 = timed(lambda: dv.frag_bcopy_batch(descs_d8, n=n - 1, mode=mode, out=out, rows_hint=args.rows_hint))
    copyd8_ok = bool(torch.equal(src[:(n - 1) * L], dst[8:8 + (n - 1) * L]))
    # byte-misaligned destinations (dst + 1)
    descs_d1 = dv.make_copy_descs(src, offs[:-1], dst, offs[:-1] + np.uint64(1), np.full(n - 1, L), np.full(n - 1, L))
    _, kern_dst1 = timed(lambda: dv.frag_bcopy_batch(descs_d1, n=n - 1, mode=mode, out=out, rows_hint=args.rows_hint))
    copyd1_ok = bool(torch.equal(src[:(n - 1) * L], dst[1:1 + (n - 1) * L]))
    _, kern_copy = timed(lambda: dst.copy_(src))
    # GM's own send shape (gm/sendFrag.cc:147-155): 65,456-byte payloads of a 1 GiB message into
    # 64 KiB ring slots right after the 72-byte header, checksums vs the read-only kernels
    gm_L, gm_stride, gm_n = 65456, 65536, min(16384, (n * L) // 65536 - 1)
    gm_msg, gm_dst = src[:gm_n * gm_L], dst[:72 + gm_n * gm_stride]
    gm_out = torch.empty(gm_n, dtype=torch.int32, device="cuda")
    gm_run = lambda: dv.msg_bcopy(gm_msg, gm_L, gm_dst[72:], gm_stride, mode=mode, out=gm_out)  # noqa: E731
    for _ in range(40):  # past the clocks' transient (profiles/r03/light_transient.txt)
        gm_run()
    _, kern_gm = timed(gm_run)
    gm_copy_ok = bool(torch.equal(gm_dst[72:72 + gm_n * gm_stride].view(gm_n, gm_stride)[:, :gm_L],
                                  gm_msg.view(gm_n, gm_L)))
    gm_same = bool(torch.equal(gm_out, dv.msg_csum(gm_msg, gm_L, mode=mode)))
    moved = 2.0 * n * L
    achieved = moved / kern / 1e9
    pow2 = L & (L - 1) == 0
    kname = ((f"sum_row4k_copy_kernel<{L // 16}> (the copy) + crc_regular_kernel<kSub = {L // 64}> (the packed-row CRC "
              "of the source)" if pow2 and 64 <= L <= 1024 and n * L >= 256 * 4096 else "crc_light_copy_kernel")
             if mode == dv.CRC32 else
             f"sum_row4k_copy_kernel<{L // 16}> (one short-lived workgroup per 4 KiB of the message)"
             if pow2 and 64 <= L <= 1024 and n * L >= 256 * 4096 else
             "sum_copy_row_kernel" if L >= 4096 else "sum_copy_wg_kernel<MsgCopySource> (one fragment per workgroup)")
    print(json.dumps({
        "metric": "device-resident fused copy+checksum GiB/s of payload (bcopy); % of HBM roofline",
        "value": round(n * L / GIB / (wall / args.steps), 2), "unit": "GiB/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": f"synthetic: splitmix64 stream seed {args.seed} (SURVEY.md 8(d)), generated on device",
        "config": {"workload": f"{n} x {L} B fragments copied into a staging array with the "
                               f"{'CRC' if mode == dv.CRC32 else 'sum'} fused (lampi_msg_bcopy)",
                   "fragments": n, "frag_bytes": L, "rows_hint": args.rows_hint},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": _traffic(f"{'crc' if mode == dv.CRC32 else 'sum'}_bcopy_{n}x{L}"),
                     "traffic_source": _traffic(f"{'crc' if mode == dv.CRC32 else 'sum'}_bcopy_{n}x{L}", "source"),
                     "kernel": kname,
                     "kernel_avg_ms": round(kern * 1e3, 4), "algorithmic_bytes_per_launch": int(moved),
                     "note": "algorithmic bytes = payload read + payload written"},
        "descriptor_batch": {"kernel_avg_ms": round(kern_desc * 1e3, 4),
                             "achieved_GBs": round(moved / kern_desc / 1e9, 1),
                             "frac": round(moved / kern_desc / 1e9 / HBM_PEAK_GBS, 4)},
        "descriptor_batch_src8": {"what": "n-1 fragments from src + 8 (payload after a 72-byte GM header) "
                                          "to aligned dst; copy checked", "kernel_avg_ms": round(kern_desc8 * 1e3, 4),
                                  "frac": round(2.0 * (n - 1) * L / kern_desc8 / 1e9 / HBM_PEAK_GBS, 4),
                                  "copy_ok": copy8_ok},
        "descriptor_batch_dst8": {"what": "n-1 fragments from aligned src to dst + 8 (gather into GM slots after a "
                                          "72-byte header); copy checked", "kernel_avg_ms": round(kern_dst8 * 1e3, 4),
                                  "frac": round(2.0 * (n - 1) * L / kern_dst8 / 1e9 / HBM_PEAK_GBS, 4),
                                  "copy_ok": copyd8_ok},
        "descriptor_batch_dst1": {"what": "n-1 fragments from aligned src to dst + 1 (byte-misaligned); copy checked",
                                  "kernel_avg_ms": round(kern_dst1 * 1e3, 4),
                                  "frac": round(2.0 * (n - 1) * L / kern_dst1 / 1e9 / HBM_PEAK_GBS, 4),
                                  "copy_ok": copyd1_ok},
        "gm_send_slots": {"what": f"{gm_n} x {gm_L} B payloads of one message into {gm_stride}-byte slots after "
                                  f"a 72-byte header (lampi_msg_bcopy, dst % 16 = 8); copy and checksums "
                                  f"(vs lampi_msg_csum) checked", "kernel": kname if mode == dv.CRC32 else
                          "sum_copy_row_kernel", "kernel_avg_ms": round(kern_gm * 1e3, 4),
                          "frac": round(2.0 * gm_n * gm_L / kern_gm / 1e9 / HBM_PEAK_GBS, 4),
                          "traffic": _traffic(f"{'crc' if mode == dv.CRC32 else 'sum'}_bcopy_gm_slots"),
                          "copy_ok": gm_copy_ok, "checksums_ok": gm_same},
        "copy_reference": {"what": "torch dst.copy_(src), same bytes, no checksum",
                           "kernel_avg_ms": round(kern_copy * 1e3, 4),
                           "achieved_GBs": round(moved / kern_copy / 1e9, 1)},
        "parity": {**parity, "descriptor_batch": parity_desc,
                   "ok_all": bool(parity["ok"] and parity_desc["ok"] and gm_copy_ok and gm_same)},
        "cpu_baseline": None}))


def run_recv(args):
    """The receive step (RecvDesc_t::CopyToApp, ref src/path/common/BaseDesc.cc:288-342) over the
    config B shape in GM receive slots: n fragments of L bytes, each behind a 72-byte gmHeaderData
    whose dataChecksum (@64) the send side stamped (slot stride 72 + L + 8), delivered into one
    contiguous application buffer with the checksum verified in the same pass
    (lampi_copy_to_app_batch).  Roofline bytes = L read + L written per fragment."""
    import numpy as np
    import torch

    from lampi_amd import device as dv
    from lampi_amd import shard

    rank, world, _ = dist_setup(args)
    if world != 1:
        raise SystemExit("--recv is a single-GPU measurement")
    n, L = args.frags, args.frag_bytes
    mode = dv.CRC32 if args.mode == "crc" else dv.SUM32
    stride = 72 + L + 8
    src = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    dv.fill_stream_frags(src, n, L, args.seed)
    nic = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    # send side: gather every fragment into its slot behind the header, checksum fused, and stamp
    # it into the header's dataChecksum (lampi_msg_bcopy + a strided store of the u32 array)
    sent = dv.msg_bcopy(src, L, nic[72:], dst_stride=stride, mode=mode)
    nic.view(n, stride)[:, 64:68].copy_(sent.view(torch.uint8).view(n, 4))
    del src
    app = torch.zeros(n * L, dtype=torch.uint8, device="cuda")
    offs = np.arange(n, dtype=np.uint64)
    descs = dv.make_recv_descs(nic, offs * np.uint64(stride) + np.uint64(72), app, offs * np.uint64(L),
                               np.full(n, L), np.full(n, 1 << 40, dtype=np.int64))
    run = lambda: dv.copy_to_app_batch(descs, nic, expected_stride=stride, expected_offset=64, n=n, mode=mode,  # noqa
                                       rows_hint=args.rows_hint)
    res = _warm(run, args.warmup)
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)  # (events at the ends of the K back-to-back calls, as timed() in run_bcopy)
    for _ in range(args.steps):
        res = run()
    e1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern = e0.elapsed_time(e1) / args.steps / 1e3
    copied, csum, mask, nbad = res
    vals = dv.as_u32(csum)
    got = shard.digest(vals, np.arange(n, dtype=np.uint64))
    want = golden_digest(args.seed, n, L, mode == dv.CRC32)
    app_ok = bool(torch.equal(app.view(n, L), nic.view(n, stride)[:, 72:72 + L]))
    # no committed digest for this shape: the checksums are unpinned (ok None), whatever the copy says
    ok = (int(nbad.item()) == 0 and bool((copied == L).all().item()) and app_ok
          and (None if want is None else got == tuple(want)))
    moved = 2.0 * n * L
    achieved = moved / kern / 1e9
    print(json.dumps({
        "metric": "device-resident batched receive step (CopyToApp: copy + checksum + CheckData), GiB/s of "
                  "payload; % of HBM roofline",
        "value": round(n * L / GIB / (wall / args.steps), 2), "unit": "GiB/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": f"synthetic: splitmix64 stream seed {args.seed} (SURVEY.md 8(d)) in GM receive slots",
        "config": {"workload": f"{n} x {L} B fragments, 72-byte gmHeaderData + payload slots (stride {stride}), "
                               f"{'CRC' if mode == dv.CRC32 else 'sum'} verified against dataChecksum, delivered "
                               "into one application buffer (lampi_copy_to_app_batch)", "fragments": n,
                   "frag_bytes": L, "rows_hint": args.rows_hint},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": _traffic(f"{'crc' if mode == dv.CRC32 else 'sum'}_recv_{n}x{L}"),
                     "traffic_source": _traffic(f"{'crc' if mode == dv.CRC32 else 'sum'}_recv_{n}x{L}", "source"),
                     "kernel": _recv_schedule(mode == dv.CRC32, L, args.rows_hint),
                     "kernel_avg_ms": round(kern * 1e3, 4), "algorithmic_bytes_per_launch": int(moved),
                     "note": "algorithmic bytes = payload read + payload written; the 4-byte expected value and "
                             "32-byte descriptor per fragment excluded"},
        "parity": {"check": "nbad == 0, every fragment fully copied, app == slot payloads, checksum digest vs "
                            "committed config digest" + ("" if want is not None else
                                                         " (none committed for this shape: unpinned)"),
                   "xor": f"{got[0]:08x}", "wsum": f"{got[1]:08x}", "ok": None if ok is None else bool(ok)},
        "cpu_baseline": None}), flush=True)


def run_recv_alternate(args):
    """The receive step on one stream that alternates two shapes: GM batches (16,384 x
    65,456-byte payloads in 64 KiB-ish slots, 1 GiB) and IB batches (262,144 x 1,976 bytes, 0.5 GiB), each from
    its own descriptor array.  The library learns a batch's shape per descriptor array (round 5), so each
    should keep the schedule it gets alone.  Reported: each shape alone without a hint (learned), GM with
    LAMPI_CSUM_ROWS_HINT(16), and each inside the alternating sequence (HIP events around every call);
    roofline bytes = payload read + written."""
    import numpy as np
    import torch

    from lampi_amd import device as dv

    rank, world, _ = dist_setup(args)
    if world != 1:
        raise SystemExit("--recv --alternate is a single-GPU measurement")
    mode = dv.CRC32 if args.mode == "crc" else dv.SUM32

    def build(n, L, seed):
        stride = 72 + L + 8
        src = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        dv.fill_stream_frags(src, n, L, seed)
        nic = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
        sent = dv.msg_bcopy(src, L, nic[72:], dst_stride=stride, mode=mode)
        nic.view(n, stride)[:, 64:68].copy_(sent.view(torch.uint8).view(n, 4))
        del src
        app = torch.zeros(n * L, dtype=torch.uint8, device="cuda")
        offs = np.arange(n, dtype=np.uint64)
        descs = dv.make_recv_descs(nic, offs * np.uint64(stride) + np.uint64(72), app, offs * np.uint64(L),
                                   np.full(n, L), np.full(n, 1 << 40, dtype=np.int64))
        return dict(n=n, L=L, stride=stride, nic=nic, app=app, descs=descs)

    gm, ib = build(16384, 65456, 7), build(262144, 1976, 8)

    def call(b, hint=0):
        return dv.copy_to_app_batch(b["descs"], b["nic"], expected_stride=b["stride"], expected_offset=64, n=b["n"],
                                    mode=mode, rows_hint=hint)

    stream = torch.cuda.current_stream()

    def alone(fn):
        _warm(fn, args.warmup)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.steps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.steps / 1e3

    t_gm_hint = alone(lambda: call(gm, 16))
    t_gm = alone(lambda: call(gm))
    t_ib = alone(lambda: call(ib))
    _warm(lambda: (call(gm), call(ib)), args.warmup)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.steps + 1)]
    ev[0].record(stream)
    for i in range(args.steps):
        call(gm)
        ev[2 * i + 1].record(stream)
        call(ib)
        ev[2 * i + 2].record(stream)
    torch.cuda.synchronize()
    a_gm = sum(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(args.steps)) / args.steps / 1e3
    a_ib = sum(ev[2 * i + 1].elapsed_time(ev[2 * i + 2]) for i in range(args.steps)) / args.steps / 1e3
    ok = True
    for b in (gm, ib):
        copied, csum, mask, nbad = call(b)
        ok = ok and int(nbad.item()) == 0 and bool((copied == b["L"]).all().item()) and bool(
            torch.equal(b["app"].view(b["n"], b["L"]), b["nic"].view(b["n"], b["stride"])[:, 72:72 + b["L"]]))
    frac = lambda b, t: round(2.0 * b["n"] * b["L"] / t / 1e9 / HBM_PEAK_GBS, 4)  # noqa: E731
    print(json.dumps({
        "metric": "device-resident batched receive step on a stream alternating GM and IB batches; % of HBM roofline",
        "value": round((gm["n"] * gm["L"] + ib["n"] * ib["L"]) / GIB / (a_gm + a_ib), 2), "unit": "GiB/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "higher_is_better": True, "dtype": "u8",
        "data": "synthetic: splitmix64 streams seeds 7 / 8 in GM / IB receive slots (72-byte header + payload)",
        "config": {"workload": "alternating lampi_copy_to_app_batch calls on one stream: 16,384 x 65,456 B (GM) and "
                               "262,144 x 1,976 B (IB), separate descriptor arrays, no hint",
                   "mode": args.mode},
        "gm": {"alone_hint16_frac": frac(gm, t_gm_hint), "alone_learned_frac": frac(gm, t_gm),
               "alternating_frac": frac(gm, a_gm), "alternating_ms": round(a_gm * 1e3, 4)},
        "ib": {"alone_learned_frac": frac(ib, t_ib), "alternating_frac": frac(ib, a_ib),
               "alternating_ms": round(a_ib * 1e3, 4)},
        "parity": {"check": "nbad == 0, every fragment fully copied, app == slot payloads (checksums verified "
                            "against the send side's, stamped by lampi_msg_bcopy)", "ok": bool(ok)},
        "cpu_baseline": None}), flush=True)


def run_latency(args):
    """Small batches: per-call time of lampi_frag_csum_batch over n 4 KiB descriptor
    fragments, three ways -- stream-ordered back-to-back calls (device time per call, HIP events),
    one call + synchronize (host round trip), and the same call replayed from a captured HIP graph.
    Results are checked against a committed digest only where one exists (the full batch)."""
    import numpy as np
    import torch

    from lampi_amd import device as dv

    rank, world, _ = dist_setup(args)
    if world != 1:
        raise SystemExit("--latency is a single-GPU measurement")
    L = 4096
    nmax = 65536
    buf = torch.empty(nmax * L, dtype=torch.uint8, device="cuda")
    dv.fill_stream_frags(buf, nmax, L, 2)
    descs = dv.make_descs(buf, np.arange(nmax, dtype=np.uint64) * L, np.full(nmax, L, np.uint64))
    out = torch.empty(nmax, dtype=torch.int32, device="cuda")
    rows = []
    for n in (1, 16, 256, 4096, 65536):
        run = lambda: dv.frag_csum_batch(descs, n=n, out=out)  # noqa: E731
        for _ in range(20):
            run()
        torch.cuda.synchronize()
        reps = 200
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        stream_us = e0.elapsed_time(e1) / reps * 1e3
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            run()
            torch.cuda.synchronize()
            t.append(time.perf_counter() - t0)
        sync_us = float(np.median(t)) * 1e6
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            run()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            for _ in range(8):  # eight batches per replay (a send loop over eight messages)
                run()
        g.replay()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps // 8):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        graph_us = e0.elapsed_time(e1) / (reps // 8 * 8) * 1e3
        rows.append({"fragments": n, "bytes": n * L, "stream_us_per_call": round(stream_us, 2),
                     "sync_round_trip_us": round(sync_us, 2), "graph_us_per_call": round(graph_us, 2),
                     "GiB_per_s_stream": round(n * L / GIB / (stream_us / 1e6), 2)})
    # the same fragments as one contiguous message (lampi_msg_csum: the regular kernel)
    msg_rows = []
    for n in (256, 4096, 65536):
        run = lambda: dv.msg_csum(buf[:n * L], L, out=out)  # noqa: E731
        for _ in range(20):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 200 * 1e3
        msg_rows.append({"fragments": n, "bytes": n * L, "stream_us_per_call": round(us, 2),
                         "GiB_per_s_stream": round(n * L / GIB / (us / 1e6), 2)})
    rows.append({"lampi_msg_csum": msg_rows})
    # the drop-in host entry points (pageable host buffer in, checksum out; pinned bounce buffer
    # inside the library): what an unchanged src/path call site pays per call
    from lampi_amd._lib import lib as _clib

    host_rows = []
    hb = np.frombuffer(np.random.default_rng(3).bytes(1 << 20), dtype=np.uint8).copy()
    hd = np.empty_like(hb)
    for nb in (1976, 4096, 65456, 1 << 20):
        t = []
        for i in range(220):
            t0 = time.perf_counter()
            _clib().lampi_uicrc(hb.ctypes.data, nb, 0xFFFFFFFF)
            t.append(time.perf_counter() - t0)
        tc = []
        for i in range(220):
            t0 = time.perf_counter()
            _clib().lampi_bcopy_uicrc(hb.ctypes.data, hd.ctypes.data, nb, nb, 0xFFFFFFFF)
            tc.append(time.perf_counter() - t0)
        ts = []
        pint, plen = ctypes.c_uint(0), ctypes.c_uint(0)
        for i in range(220):
            t0 = time.perf_counter()
            _clib().lampi_uicsum(hb.ctypes.data, nb, ctypes.byref(pint), ctypes.byref(plen))
            ts.append(time.perf_counter() - t0)
        host_rows.append({"bytes": nb, "uicrc_us_median": round(float(np.median(t[20:])) * 1e6, 2),
                          "bcopy_uicrc_us_median": round(float(np.median(tc[20:])) * 1e6, 2),
                          "uicsum_us_median": round(float(np.median(ts[20:])) * 1e6, 2)})
    rows.append({"host_entry_points": host_rows})
    dv.frag_csum_batch(descs, n=nmax, out=out)
    got = dv.as_u32(out[:nmax])
    from lampi_amd import shard

    digest = shard.digest(got, np.arange(nmax, dtype=np.uint64))
    print(json.dumps({"metric": "small-batch latency of lampi_frag_csum_batch (4 KiB CRC descriptors)",
                      "unit": "us", "results": rows, "last_batch_xor": f"{digest[0]:08x}"}), flush=True)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if args.latency:
        run_latency(args)
        return
    if args.bcopy:
        run_bcopy(args)
        return
    if args.recv and args.alternate:
        run_recv_alternate(args)
        return
    if args.recv:
        run_recv(args)
        return
    if args.e2e:
        run_e2e(args)
        return
    if args.config == "C":
        run_mixed(args)
        return
    rank, world, result = run_device(args)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    if result is not None and not result["parity"]["all_ranks_ok"]:
        sys.exit(3)  # a rank's checksums differ from the committed digests


if __name__ == "__main__":
    main()
