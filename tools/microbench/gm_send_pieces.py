"""GM's own send shape -- 16,384 payloads of 65,456 bytes gathered into 64 KiB slots (payload at
+72) with the checksum fused -- through lampi_msg_bcopy (one wave walks a whole fragment) and through
lampi_chain_csum_batch with every fragment cut into 4 KiB pieces (adjacent pieces go to adjacent
waves; the per-piece checksums are folded per fragment afterwards).

python tools/microbench/gm_send_pieces.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lampi_amd import device as dv  # noqa: E402

L, n, stride, off, P = 65456, 1 << 14, 65536, 72, 4096
msg = torch.empty(n * L, dtype=torch.uint8, device="cuda")
dv.fill_stream(msg, seed=13)
dst = torch.zeros(off + n * stride, dtype=torch.uint8, device="cuda")
npf = (L + P - 1) // P
k = np.repeat(np.arange(n, dtype=np.uint64), npf)
j = np.tile(np.arange(npf, dtype=np.uint64), n)
so = k * np.uint64(L) + j * np.uint64(P)
ln = np.minimum(np.uint64(P), np.uint64(L) - j * np.uint64(P))
do = np.uint64(off) + k * np.uint64(stride) + j * np.uint64(P)
pieces = dv.make_copy_descs(msg, so, dst, do, ln, ln)
first = np.arange(n + 1, dtype=np.uint32) * npf


def timed(fn, reps=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


for mode, name in ((dv.CRC32, "crc"), (dv.SUM32, "sum")):
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    s1 = timed(lambda: dv.msg_bcopy(msg, L, dst[off:], stride, mode=mode, out=out))
    ref = dv.as_u32(out).copy()
    s2 = timed(lambda: dv.chain_csum_batch(pieces, first, mode=mode, out=out))
    same = bool(np.array_equal(dv.as_u32(out), ref))
    print(f"{name}: msg_bcopy {2 * n * L / s1 / 8e12:.3f}, 4 KiB pieces + fold {2 * n * L / s2 / 8e12:.3f} of 8 TB/s "
          f"(read + write), same checksums {same}", flush=True)
