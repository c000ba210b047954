"""SUM fused copies of large message fragments (lampi_msg_bcopy, LA-MPI's default mode): read +
write fraction of 8 TB/s into GM-style slots (payload at +72 of 64 KiB slots) and into a
contiguous destination, checksums checked against lampi_msg_csum of the same message.

python tools/microbench/sum_copy_rows.py   (LAMPI_CSUM_LIB selects the library under test)
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

from lampi_amd import device as dv  # noqa: E402


def timed(run, reps=10):
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


for gib in (1, 8):
    for L in (16384, 65456, 65536):
        n = (gib << 30) // L
        msg = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        dv.fill_stream(msg, seed=21)
        ref = dv.as_u32(dv.msg_csum(msg, L, mode=dv.SUM32))
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        for stride, off in ((max(L, 65536) if L > 16384 else L + 80, 72), (L, 0)):
            dst = torch.zeros(off + n * stride, dtype=torch.uint8, device="cuda")
            s = timed(lambda: dv.msg_bcopy(msg, L, dst[off:], stride, mode=dv.SUM32, out=out))
            ok = (dv.as_u32(out) == ref).all() and torch.equal(dst[off:off + n * stride].view(n, stride)[:, :L],
                                                                msg.view(n, L))
            print(f"{gib:2d} GiB L={L} stride {stride} +{off:<2d} sum copy {2 * n * L / s / 8e12:.3f} of 8 TB/s, ok {bool(ok)}",
                  flush=True)
            del dst
        del msg, out
