"""Descriptor batches of large uniform fragments (lampi_frag_csum_batch), on the default count split and
with LAMPI_CSUM_BY_BYTES (below 32,768 descriptors: plan_kernel + the piece streams over segments).
Reports the fraction of the 8 TB/s HBM-read roofline per shape and checks every batch against
lampi_msg_csum over the same bytes (an independent kernel).  "rows": LAMPI_CSUM_ROWS_HINT(R), R the
fragments' row count (row segments computed on the device).
python tools/microbench/bigdesc_scan.py [crc|sum]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lampi_amd import device as dv  # noqa: E402

mode = dv.SUM32 if len(sys.argv) > 1 and sys.argv[1] == "sum" else dv.CRC32
buf = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
dv.fill_stream(buf, seed=9)


def timed(fn, reps=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


for total, L in ((1 << 30, 65456), (1 << 30, 65536), (1 << 30, 262144), (1 << 30, 1 << 20), (1 << 30, 4 << 20),
                 (4 << 30, 65456), (4 << 20, 4 << 20), (16 << 20, 4 << 20), (64 << 20, 16 << 20), (16 << 20, 4096),
                 (1 << 20, 4096), (4096, 4096)):
    n = total // L
    d = dv.make_descs(buf, np.arange(n, dtype=np.uint64) * np.uint64(L), np.full(n, L, np.uint64))
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    ref = dv.msg_csum(buf[:n * L], L, mode=mode)
    R = (L + 4095) // 4096
    for split, by_bytes, hint in (("count   ", False, 0), ("by_bytes", True, 0), ("rows    ", False, min(R, 4095))):
        if split.startswith("rows") and R < 2:
            continue
        t = timed(lambda: dv.frag_csum_batch(d, n=n, out=out, mode=mode, by_bytes=by_bytes, rows_hint=hint))
        ok = bool(torch.equal(out, ref))
        print(f"{'crc' if mode == dv.CRC32 else 'sum'} {split} descriptors L={L:8d} "
              f"n={n:6d} {n * L / 2**20:8.1f} MiB {t * 1e6:9.2f} us  {n * L / t / 8e12:.3f} of 8 TB/s  "
              f"same_as_msg_csum={ok}", flush=True)
