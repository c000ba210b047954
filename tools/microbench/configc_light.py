"""Config C (4 GiB of Zipf-sized fragments, 64 B..64 KiB) through lampi_frag_csum_batch with and
without LAMPI_CSUM_ROWS_HINT(r): r >= 8 runs every fragment on the read-only table-light kernel (one
wave per fragment), r < 8 the piece streams.  Fraction of 8 TB/s over the bytes read; results must
match the plain batch.  python tools/microbench/configc_light.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lampi_amd import device as dv  # noqa: E402
from lampi_amd.workload import zipf_lengths  # noqa: E402


def timed(fn, reps=20):
    for _ in range(200):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


lens = zipf_lengths(4 << 30)
offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
total = int(lens.sum(dtype=np.uint64))
buf = torch.empty(total, dtype=torch.uint8, device="cuda")
dv.fill_stream(buf, seed=5)
descs = dv.make_descs(buf, offs, lens)
want = dv.frag_csum_batch(descs, mode=dv.CRC32).clone()
rows = (lens + 4095) // 4096
for lo in (1, 2, 4, 8, 16):
    sel = rows >= lo
    print(f"fragments of >= {lo:2d} rows: {sel.mean():.3f} of the count, "
          f"{lens[sel].sum(dtype=np.uint64) / total:.3f} of the bytes", flush=True)
out = torch.empty_like(want)
for h in (0, 8, 16):
    s = timed(lambda: dv.frag_csum_batch(descs, mode=dv.CRC32, out=out, rows_hint=h))
    print(f"config C hint={h:3d} {total / s / 8e12:.3f} of 8 TB/s ok={torch.equal(out, want)} n={lens.size}",
          flush=True)
