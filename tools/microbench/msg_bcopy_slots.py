"""Time lampi_msg_bcopy into GM-style slots (payload after a 72-byte header: dst % 16 = 8).

python tools/microbench/msg_bcopy_slots.py  (LAMPI_CSUM_LIB selects the library under test)
Prints GB/s of read + write and the fraction of the 8 TB/s roofline per mode.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

from lampi_amd import device as dv  # noqa: E402

for L, n, stride, off in ((4096, 1 << 20, 4096 + 80, 72),   # 4 KiB payloads in 4,176-byte slots
                          (65456, 1 << 14, 65536, 72)):      # GM's own: 65,456-byte payloads in 64 KiB slots
    msg = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    dv.fill_stream(msg, seed=13)
    dst = torch.zeros(off + n * stride, dtype=torch.uint8, device="cuda")
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    for mode, name in ((dv.CRC32, "crc"), (dv.SUM32, "sum")):
        run = lambda: dv.msg_bcopy(msg, L, dst[off:], stride, mode=mode, out=out)  # noqa: E731
        for _ in range(40):  # past the clocks' transient (a dip over the first ~20 calls: profiles/r03/light_transient.txt)
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(30):
            run()
        e1.record()
        torch.cuda.synchronize()
        s = e0.elapsed_time(e1) / 30 / 1e3
        ok = torch.equal(dst[off:off + n * stride].view(n, stride)[:, :L], msg.view(n, L))
        same = torch.equal(out, dv.msg_csum(msg, L, mode=mode))  # the read-only kernels, an independent path
        print(f"L={L} slot={stride} {name}: {2 * n * L / s / 1e9:.1f} GB/s = {2 * n * L / s / 8e12:.3f} of 8 TB/s, "
              f"copy ok {ok}, checksums = msg_csum {same}", flush=True)
    del msg, dst, out
