"""Read-only CRC of descriptor batches: the piece streams (lampi_frag_csum_batch, with and without
LAMPI_CSUM_ROWS_HINT) against the table-light copy kernel run with copylen 0 and one row group per
row (lampi_frag_bcopy_batch, rows_hint = R).  1 GiB of L-byte fragments; fraction of 8 TB/s over the
bytes read.  python tools/microbench/desc_readonly_light.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lampi_amd import device as dv  # noqa: E402


def timed(fn, reps=20):
    for _ in range(40):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


src = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
dv.fill_stream(src, seed=31)
dst = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
for L in (4096, 16384, 65456, 65536, 1 << 20, 4 << 20):
    n = (1 << 30) // L
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    want = dv.msg_csum(src[:n * L], L, mode=dv.CRC32)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    R = (L + 4095) // 4096
    descs = dv.make_descs(src, offs, np.full(n, L))
    for h in (0, R):
        s = timed(lambda: dv.frag_csum_batch(descs, n=n, out=out, mode=dv.CRC32, rows_hint=h))
        print(f"streams L={L:8d} n={n:6d} hint={h:4d} {n * L / s / 8e12:.3f} of 8 TB/s  ok={torch.equal(out, want)}",
              flush=True)
    cd = dv.make_copy_descs(src, offs, dst, np.zeros(n, dtype=np.uint64), np.zeros(n), np.full(n, L))
    for h in sorted({1, R, min(R, 16)}):
        out.fill_(-1)
        s = timed(lambda: dv.frag_bcopy_batch(cd, n=n, out=out, mode=dv.CRC32, rows_hint=h))
        print(f"light   L={L:8d} n={n:6d} hint={h:4d} {n * L / s / 8e12:.3f} of 8 TB/s  ok={torch.equal(out, want)}",
              flush=True)
