"""Read-only message checksums (lampi_msg_csum, CRC) by fragment length and batch size: where the
regular kernel (uniform fragments of whole 4 KiB rows) stops paying and how the work split
behaves for large fragments.  16 GiB buffer, prefixes of 1 / 4 / 16 GiB.

python tools/microbench/bigfrag_scan.py [--quick] [--lens L1,L2,...]   (--quick: 1 and 16 GiB only)
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


big = torch.empty(16 << 30, dtype=torch.uint8, device="cuda")
dv.fill_stream(big, seed=3)
totals = (1 << 30, 16 << 30) if "--quick" in sys.argv else (1 << 30, 4 << 30, 16 << 30)
lens = (4096, 16384, 32768, 65536, 65456, 262144)
if "--lens" in sys.argv:
    lens = tuple(int(x) for x in sys.argv[sys.argv.index("--lens") + 1].split(","))
for L in lens:
    for tot in totals:
        n = tot // L
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        for mode, name in ((dv.CRC32, "crc"), (dv.SUM32, "sum")):
            s = timed(lambda: dv.msg_csum(big, L, mode=mode, out=out, msg_len=n * L))
            print(f"L={L:6d} total {tot >> 30:2d} GiB n={n:8d} {name} read {n * L / s / 8e12:.3f}", flush=True)
