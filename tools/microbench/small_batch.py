"""Read-only descriptor batches of FEW fragments (lampi_frag_csum_batch under the learned-shape minimum of
256 fragments): the default schedule, the byte-balanced plan (LAMPI_CSUM_BY_BYTES) and the caller's rows
hint, per call in microseconds and as a fraction of the 8 TB/s roofline.

python tools/microbench/small_batch.py
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


SHAPES = [(16, 16 << 20), (64, 4 << 20), (200, 1 << 20), (16, 1 << 20), (100, 65456), (250, 65456),
          (100, 16384), (200, 4096), (100, 1024), (1, 64 << 20), (4, 1 << 20)]
if "--shapes" in sys.argv:
    SHAPES = [tuple(int(v) for v in s.split("x")) for s in sys.argv[sys.argv.index("--shapes") + 1].split(",")]
base = torch.empty(max(n * (L + 64) for n, L in SHAPES) + 64, dtype=torch.uint8, device="cuda")
dv.fill_stream(base, seed=5)
host = None
for n, L in SHAPES:
    offs = (np.arange(n, dtype=np.uint64) * np.uint64(L + 64)) + np.uint64(8)
    lens = np.full(n, L, np.uint64)
    descs = dv.make_descs(base, offs, lens)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    R = (L + 4095) // 4096
    for mode, name in ((dv.CRC32, "crc"), (dv.SUM32, "sum")):
        ref = dv.as_u32(dv.frag_csum_batch(descs, mode=mode, by_bytes=True)).copy()
        row = []
        for tag, kw in (("default", {}), ("by_bytes", {"by_bytes": True}),
                        ("hint", {"rows_hint": min(R, 4095)} if R > 1 else None)):
            if kw is None:
                continue
            got = dv.as_u32(dv.frag_csum_batch(descs, mode=mode, out=out, **kw))
            assert np.array_equal(got, ref), (n, L, name, tag)
            s = timed(lambda: dv.frag_csum_batch(descs, mode=mode, out=out, **kw))
            row.append(f"{tag} {s * 1e6:8.1f} us {n * L / s / 8e12:6.3f}")
        print(f"{n:4d} x {L:9d} {name}  " + "  ".join(row), flush=True)
