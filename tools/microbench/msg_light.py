"""Read-only CRC of messages cut into long fragments (lampi_msg_csum): 1 GiB and 4 GiB at GM's
65,456 bytes, 64 KiB, 131,056 bytes and 1 MiB, fraction of 8 TB/s over the bytes read; results
compared with the descriptor batch over the same fragments.  python tools/microbench/msg_light.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lampi_amd import device as dv  # noqa: E402


def timed(fn, reps=20):
    for _ in range(60):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


src = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
dv.fill_stream(src, seed=41)
for total in (64 << 20, 1 << 30, 4 << 30):
    for L in (65456, 65536, 131056, 1 << 20):
        n = total // L
        m = src[:n * L]
        want = dv.as_u32(dv.frag_csum_batch(dv.make_descs(src, np.arange(n, dtype=np.uint64) * np.uint64(L),
                                                           np.full(n, L, np.uint64), np.full(n, 0xFFFFFFFF, np.uint64))))
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        s = timed(lambda: dv.msg_csum(m, L, mode=dv.CRC32, out=out))
        ok = np.array_equal(dv.as_u32(out), want)
        print(f"msg {total >> 20:5d} MiB L={L:8d} n={n:6d} {n * L / s / 8e12:.3f} of 8 TB/s  ok={ok}", flush=True)
