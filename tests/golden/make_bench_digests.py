#!/usr/bin/env python3
"""Generate tests/golden/bench_digests.json: oracle digests of the uniform batches bench.py runs.

bench.py checks its results against committed data only (the oracle is not imported on the
measured path).  Each entry is the digest (XOR, sum of c_k*(2k+1) mod 2^32) of
fragments k = 0 .. n_total-1 of stream `seed` at L bytes, as the oracle (oracle/csum_ref.c)
computes them; a weak-scaled N-GPU run of bench.py covers n_total = N x fragments-per-GPU
(rank r holds k = r mod N) and combines the per-rank digests (lampi_amd/shard.py).

Shard entries (`nshard`, `shard` keys) cover only k = shard (mod nshard) of the n_total
fragments, with the global k in the weighted sum: BASELINE config D's per-GPU shards
(seed 3, 32M x 16 KiB, 8 GPUs), whose CRC XORs BASELINE.md lists from the compiled reference
(the generator checks its XORs against those before writing).

Existing entries are kept; only missing ones are computed.
Run in the build container (8 threads; config D shards ~8 min):
    python tests/golden/make_bench_digests.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle.oracle import Restatement  # noqa: E402

# (seed, fragments per GPU, L, mode, GPU counts)
CASES = [
    (2, 4194304, 4096, 0, (1, 2, 4, 8)),   # config B, the default bench line, weak-scaled
    (2, 4194304, 4096, 1, (1, 2, 4, 8)),   # the same in SUM mode (--mode sum)
    (2, 1048576, 16384, 0, (1,)),          # --frags 1048576 --frag-bytes 16384
    (2, 1048576, 16384, 1, (1,)),
    (1, 1048576, 1024, 0, (1,)),           # config A shape
    (2, 16404, 65456, 0, (1,)),            # --desc: GM's payloads (--rows-hint 16), 1 GiB
    (2, 16404, 65456, 1, (1,)),
    (2, 1024, 1048576, 0, (1,)),           # --desc --rows-hint 256 / 1024: 1 MiB and 4 MiB fragments
    (2, 256, 4194304, 0, (1,)),
    (2, 16384, 65456, 0, (1,)),            # --recv --frags 16384 --frag-bytes 65456: the GM receive lines
    (2, 16384, 65456, 1, (1,)),
    (2, 1024, 1048576, 1, (1,)),           # --desc --mode sum, 1 MiB / 4 MiB
    (2, 256, 4194304, 1, (1,)),
    (1, 1048576, 1024, 1, (1,)),           # config A shape in SUM mode (round 6: packed rows)
    (2, 16777216, 64, 0, (1,)),            # --frags 16777216 --frag-bytes 64: 1 GiB of 64-byte fragments
    (2, 16777216, 64, 1, (1,)),
    (2, 4194304, 256, 0, (1,)),            # 1 GiB of 256-byte fragments
    (2, 4194304, 256, 1, (1,)),
    (2, 2097152, 512, 0, (1,)),            # 1 GiB of 512-byte fragments
    (2, 2097152, 512, 1, (1,)),
]
# config D per-GPU shards: (seed, n_total, L, mode, nshard)
SHARD_CASES = [(3, 33554432, 16384, 0, 8), (3, 33554432, 16384, 1, 8)]
# CRC XOR of GPU g's shard (computed there from the compiled reference)
CONFIG_D_SHARD_XOR = [0x54862C49, 0x046DA633, 0x53ABB493, 0xEB1A2E44, 0xB9EACC67, 0x0BEC3926, 0x937B2402, 0x3B821C43]


def key(e):
    return (e["seed"], e["n_total"], e["frag_bytes"], e["mode"], e.get("nshard", 1), e.get("shard", 0))


def main():
    ref = Restatement()
    path = os.path.join(ROOT, "tests", "golden", "bench_digests.json")
    try:
        with open(path) as f:
            out = json.load(f)["entries"]
    except (OSError, ValueError, KeyError):
        out = []
    have = {key(e) for e in out}
    todo = [(seed, n * g, L, mode, 1, 0) for seed, n, L, mode, gpus in CASES for g in gpus]
    todo += [(seed, n, L, mode, ns, s) for seed, n, L, mode, ns in SHARD_CASES for s in range(ns)]
    for seed, n, L, mode, ns, s in todo:
        e = {"seed": seed, "n_total": n, "frag_bytes": L, "mode": "crc" if mode == 0 else "sum"}
        if ns > 1:
            e.update(nshard=ns, shard=s)
        if key(e) in have:
            continue
        t = time.time()
        x, w = ref.uniform_digest(seed, n, L, mode, nshard=ns, shard=s, nthreads=os.cpu_count())
        if ns == 8 and seed == 3 and mode == 0 and x != CONFIG_D_SHARD_XOR[s]:
            raise SystemExit(f"shard {s}: XOR {x:08x} differs from BASELINE.md {CONFIG_D_SHARD_XOR[s]:08x}")
        e.update(xor=x, wsum=w)
        out.append(e)
        print(f"{e}: ({time.time() - t:.1f} s)", flush=True)
    with open(path, "w") as f:
        json.dump({"generator": "tests/golden/make_bench_digests.py (oracle/csum_ref.c uniform_digest)",
                   "digest": "xor, sum c_k*(2k+1) mod 2^32 over k = 0..n_total-1 (SURVEY.md 8(d)); "
                             "shard entries: only k = shard (mod nshard), global k in the weights",
                   "entries": out}, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
