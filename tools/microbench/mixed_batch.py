"""Read-only descriptor batches mixing a few huge fragments into many small ones (lampi_frag_csum_batch):
the default schedule against the byte-balanced plan (LAMPI_CSUM_BY_BYTES), per call in microseconds and
as a fraction of the 8 TB/s roofline; results checked equal.

python tools/microbench/mixed_batch.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lampi_amd import device as dv  # noqa: E402


def timed(run, reps=20):
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


MiB = 1 << 20
# (fragments, small-length bound, huge fragments, huge length)
CASES = [(1000, 600, 6, 8 * MiB), (5000, 600, 6, 8 * MiB), (5000, 16384, 2, 64 * MiB), (50000, 16384, 4, 16 * MiB),
         (300, 4096, 1, 64 * MiB), (20000, 65536, 8, 4 * MiB)]
rng = np.random.default_rng(9)
for n, small, k, big in CASES:
    lens = rng.integers(0, small, size=n).astype(np.uint64)
    lens[rng.choice(n, size=k, replace=False)] = big
    offs = (np.concatenate([[0], np.cumsum(lens)[:-1]]) + np.uint64(8)).astype(np.uint64)
    base = torch.empty(int((offs + lens).max()) + 64, dtype=torch.uint8, device="cuda")
    dv.fill_stream(base, seed=n)
    descs = dv.make_descs(base, offs, lens)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    tot = int(lens.sum())
    for mode, name in ((dv.CRC32, "crc"), (dv.SUM32, "sum")):
        ref = dv.as_u32(dv.frag_csum_batch(descs, mode=mode, by_bytes=True)).copy()
        row = []
        for tag, kw in (("default", {}), ("by_bytes", {"by_bytes": True})):
            got = dv.as_u32(dv.frag_csum_batch(descs, mode=mode, out=out, **kw))
            assert np.array_equal(got, ref), (n, name, tag)
            s = timed(lambda: dv.frag_csum_batch(descs, mode=mode, out=out, **kw))
            row.append(f"{tag} {s * 1e6:8.1f} us {tot / s / 8e12:6.3f}")
        print(f"n={n:6d} small<{small:6d} {k} x {big >> 20:3d} MiB ({tot / MiB:7.1f} MiB) {name}  " + "  ".join(row),
              flush=True)
    del base, descs
