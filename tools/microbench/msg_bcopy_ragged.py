"""CRC lampi_msg_bcopy of messages the table-light message copy does not take (fragments under 4 KiB
or not a multiple of 16 bytes, unaligned messages): 1 GiB each, fraction of 8 TB/s (read + write)
after a warm-up; copies and checksums (vs lampi_msg_csum) checked.
python tools/microbench/msg_bcopy_ragged.py  (LAMPI_CSUM_LIB picks the library)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

from lampi_amd import device as dv  # noqa: E402

buf = torch.empty((1 << 30) + 64, dtype=torch.uint8, device="cuda")
dv.fill_stream(buf, seed=41)
dst = torch.zeros((1 << 30) + (1 << 26), dtype=torch.uint8, device="cuda")
for L, stride, src_off, dst_off, what in ((1976, 2048, 0, 72, "IB 1,976-byte payloads into 2 KiB slots after 72 B"),
                                          (1976, 1976, 0, 0, "IB payloads packed"),
                                          (4099, 4176, 0, 72, "4,099-byte fragments into slots"),
                                          (65456, 65536, 3, 72, "GM payloads from a message at +3"),
                                          (16384, 16464, 8, 72, "16 KiB fragments from a message at +8")):
    n = (1 << 30) // stride
    msg = buf[src_off:src_off + n * L]
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    run = lambda: dv.msg_bcopy(msg, L, dst[dst_off:], stride, out=out)  # noqa: E731
    for _ in range(30):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        run()
    e1.record()
    torch.cuda.synchronize()
    s = e0.elapsed_time(e1) / 20 / 1e3
    ok = torch.equal(out, dv.msg_csum(msg, L)) and torch.equal(
        dst[dst_off:dst_off + n * stride].view(n, stride)[:, :L], msg.view(n, L))
    print(f"L={L:6d} stride={stride:6d} src+{src_off} dst+{dst_off}: {2 * n * L / s / 8e12:.3f} of 8 TB/s ok={ok}  "
          f"({what})", flush=True)
