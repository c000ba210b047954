#!/usr/bin/env python3
"""Generate tests/golden/bench_digests.json: oracle digests of the uniform batches bench.py runs.

bench.py checks its results against committed data only (the oracle is not imported on the
measured path).  Each entry is the digest (XOR, sum of c_k*(2k+1) mod 2^32) of
fragments k = 0 .. n_total-1 of stream `seed` at L bytes, as the oracle (oracle/csum_ref.c)
computes them; a weak-scaled N-GPU run of bench.py covers n_total = N x fragments-per-GPU
(rank r holds k = r mod N) and combines the per-rank digests (lampi_amd/shard.py).

Run in the build container (8 threads, ~6 min):  python tests/golden/make_bench_digests.py
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
]


def main():
    ref = Restatement()
    out = []
    for seed, n, L, mode, gpus in CASES:
        for g in gpus:
            t = time.time()
            x, s = ref.uniform_digest(seed, n * g, L, mode, nthreads=os.cpu_count())
            out.append({"seed": seed, "n_total": n * g, "frag_bytes": L, "mode": "crc" if mode == 0 else "sum",
                        "xor": x, "wsum": s})
            print(f"seed {seed} n {n * g} L {L} mode {mode}: {x:08x} {s:08x} ({time.time() - t:.1f} s)", flush=True)
    path = os.path.join(ROOT, "tests", "golden", "bench_digests.json")
    with open(path, "w") as f:
        json.dump({"generator": "tests/golden/make_bench_digests.py (oracle/csum_ref.c uniform_digest)",
                   "digest": "xor, sum c_k*(2k+1) mod 2^32 over k = 0..n_total-1 (SURVEY.md 8(d))",
                   "entries": out}, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
