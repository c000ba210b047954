"""SUM fused copies (bcopy_uicsum descriptor batches) by fragment size: GB/s of read + write.

python tools/microbench/sum_copy_sizes.py  (LAMPI_CSUM_LIB selects the library under test)
Each line: L bytes per fragment, n fragments (1 GiB of payload, contiguous source and destination),
16-byte-aligned and +1 destinations; the copy and the checksums are checked against the same
batch from sum_rows-free references (the source bytes, and the first run's checksums).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

from lampi_amd import device as dv  # noqa: E402

TOTAL = 1 << 30
for L in (64, 256, 1024, 1976, 4096, 16384, 65456):
    n = TOTAL // L
    src = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    dv.fill_stream(src, seed=21)
    dst = torch.zeros(n * L + 64, dtype=torch.uint8, device="cuda")
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    ref = None
    for doff in (0, 1):
        descs = dv.make_copy_descs(src, offs, dst, offs + np.uint64(doff), np.full(n, L), np.full(n, L))
        run = lambda: dv.frag_bcopy_batch(descs, mode=dv.SUM32, out=out)  # noqa: E731
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            run()
        e1.record()
        torch.cuda.synchronize()
        s = e0.elapsed_time(e1) / 10 / 1e3
        ok = torch.equal(dst[doff:doff + n * L], src)
        if ref is None:
            ref = out.clone()
        ok = ok and torch.equal(out, ref)
        print(f"L={L} n={n} dst+{doff}: {2 * n * L / s / 1e9:.1f} GB/s = {2 * n * L / s / 8e12:.3f} of 8 TB/s, "
              f"{s * 1e3:.3f} ms, ok {ok}", flush=True)
    del src, dst, out
