"""Destination alignment against the table-light CRC copy (lampi_msg_bcopy, 4 KiB fragments):
packed or slotted destinations at byte offsets 0/4/8/16/64/72 from a 256-byte boundary.
python tools/microbench/light_align.py  (prints GB/s of read + write and the fraction of 8 TB/s)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

from lampi_amd import device as dv  # noqa: E402

L, n = 4096, 1 << 20
msg = torch.empty(n * L, dtype=torch.uint8, device="cuda")
dv.fill_stream(msg, seed=13)
out = torch.empty(n, dtype=torch.int32, device="cuda")
want = dv.msg_csum(msg, L)
for stride in (4096, 4176, 4224, 8192) * 2:  # twice: the first pass includes clock ramp-up
    dst = torch.zeros(256 + n * stride, dtype=torch.uint8, device="cuda")
    for off in (0, 4, 8, 16, 64, 72):
        run = lambda: dv.msg_bcopy(msg, L, dst[off:], stride, mode=dv.CRC32, out=out)  # noqa: E731
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
        print(f"stride {stride} off {off:3d}: {2 * n * L / s / 1e9:7.1f} GB/s = {2 * n * L / s / 8e12:.3f}, "
              f"checksums ok {torch.equal(out, want)}", flush=True)
    del dst
