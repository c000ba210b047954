"""GM's send shape (65,456-byte payloads) by parts: lampi_msg_bcopy into 64 KiB slots at the
header offset 72 (dst % 16 = 8) against the same copy into slots at offset 80 / 64 (dst 16-byte
aligned) and into a contiguous destination, and lampi_msg_csum alone (no copy); 64 KiB fragments
(a whole number of 4 KiB rows: the regular kernel's copy) for comparison.  1 GiB messages.

python tools/microbench/gm_send_shapes.py [--gib G]   (message size, default 1 GiB)
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

from lampi_amd import device as dv  # noqa: E402


def timed(run, reps=20):
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


GIB = int(sys.argv[sys.argv.index("--gib") + 1]) if "--gib" in sys.argv else 1
for L in (65456, 65536):
    n = (GIB << 30) // L
    msg = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    dv.fill_stream(msg, seed=13)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    for mode, name in ((dv.CRC32, "crc"), (dv.SUM32, "sum")):
        s = timed(lambda: dv.msg_csum(msg, L, mode=mode, out=out))
        print(f"L={L} {name} msg_csum (read only)        {n * L / s / 8e12:.3f} of 8 TB/s", flush=True)
        for stride, off in ((65536, 72), (65536, 80), (65536, 64), (L, 0), (L, 8)):
            dst = torch.zeros(off + n * stride, dtype=torch.uint8, device="cuda")
            s = timed(lambda: dv.msg_bcopy(msg, L, dst[off:], stride, mode=mode, out=out))
            ok = torch.equal(dst[off:off + n * stride].view(n, stride)[:, :L], msg.view(n, L))
            print(f"L={L} {name} msg_bcopy stride {stride} +{off:<3d} {2 * n * L / s / 8e12:.3f} of 8 TB/s "
                  f"(read + write), copy ok {ok}", flush=True)
            del dst
    del msg, out
