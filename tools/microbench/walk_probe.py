"""Read-only CRC of messages with fragments that are not whole 4 KiB rows (lampi_msg_csum: the row
walker, crc_walk_kernel, where it applies): GB/s and fraction of 8 TB/s per shape, after a warm-up
past the clocks' transient.  Checksums are compared with the descriptor path (lampi_frag_csum_batch,
an independent kernel).  python tools/microbench/walk_probe.py  (LAMPI_CSUM_LIB picks the library)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lampi_amd import device as dv  # noqa: E402

buf = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
dv.fill_stream(buf, seed=21)
for L, total in ((65456, 1 << 30), (65456, 4 << 30), ((1 << 20) + 48, 1 << 30), (12288 + 80, 1 << 30),
                 (4 * 1048576 + 16, 1 << 30)):
    n = total // L
    msg = buf[:n * L]
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    run = lambda: dv.msg_csum(msg, L, out=out)  # noqa: E731
    for _ in range(40):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(30):
        run()
    e1.record()
    torch.cuda.synchronize()
    s = e0.elapsed_time(e1) / 30 / 1e3
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    descs = dv.make_descs(msg, offs, np.full(n, L))
    same = torch.equal(out, dv.frag_csum_batch(descs))
    print(f"L={L:8d} n={n:6d} {n * L / 2**20:7.1f} MiB  {s * 1e6:8.1f} us  {n * L / s / 8e12:.3f} of 8 TB/s  "
          f"same_as_descriptors={same}", flush=True)
