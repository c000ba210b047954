#!/usr/bin/env python3
"""Generate tests/golden/config_b_head.json: the per-fragment CRC and SUM of config B's first
1024 fragments (seed 2, 4 KiB), computed by the compiled reference (oracle/_ref: the
reference's own src/util/MemFunctions.cc, `uicrc(p, len)` and `uicsum(p, len)`).

bench.py --dry-run (the CPU rehearsal of the multi-rank launch, tests/test_bench_launch.py)
takes its per-rank "checksums" from this file, so that the launch, shard partition, per-rank
gather and digest combination run without a GPU and without the oracle on bench.py's path.

Run in the build container:  python tests/golden/make_head_fixture.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle.oracle import Reference, digest, splitmix_stream  # noqa: E402

SEED, N, L = 2, 1024, 4096


def main():
    ref = Reference()
    buf = splitmix_stream(SEED, 0, N * L)
    crc = [ref.uicrc(buf[k * L:(k + 1) * L]) for k in range(N)]
    sums = [ref.uicsum(buf[k * L:(k + 1) * L])[0] for k in range(N)]
    import numpy as np

    out = {"generator": "tests/golden/make_head_fixture.py (oracle/_ref: reference uicrc/uicsum)",
           "seed": SEED, "n": N, "frag_bytes": L, "crc": crc, "sum": sums,
           "digest_crc": list(digest(np.array(crc, dtype=np.uint32))),
           "digest_sum": list(digest(np.array(sums, dtype=np.uint32)))}
    if crc[:4] != [0x9AFF1C82, 0xCF9217CF, 0x84A13B32, 0x66922667]:  # BASELINE.md config B crc[0..3]
        raise SystemExit("reference CRCs differ from BASELINE.md config B crc[0..3]")
    path = os.path.join(ROOT, "tests", "golden", "config_b_head.json")
    with open(path, "w") as f:
        json.dump(out, f)
    print("wrote", path)


if __name__ == "__main__":
    main()
