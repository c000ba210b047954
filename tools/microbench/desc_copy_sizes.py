"""CRC fused copies of descriptor batches by fragment size (lampi_frag_bcopy_batch): 1 GiB of
fragments of L bytes, aligned or into destinations 8 bytes past a 16-byte boundary, and the receive
step (lampi_copy_to_app_batch) from GM-style slots.  Prints the fraction of 8 TB/s (read + write)
after a warm-up past the clocks' transient; checksums are compared with lampi_msg_csum.
python tools/microbench/desc_copy_sizes.py [crc|sum] [L,L,...]  (LAMPI_CSUM_LIB picks the library)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lampi_amd import device as dv  # noqa: E402


def timed(fn, reps=20):
    for _ in range(30):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


MODE = dv.SUM32 if len(sys.argv) > 1 and sys.argv[1] == "sum" else dv.CRC32
src = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
dv.fill_stream(src, seed=31)
dst = torch.zeros((1 << 30) + (1 << 24), dtype=torch.uint8, device="cuda")
SIZES = tuple(int(x) for x in sys.argv[2].split(",")) if len(sys.argv) > 2 else (1976, 4096, 16384, 65456, 1 << 20)
for L in SIZES:
    n = (1 << 30) // (L + 80)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    want = dv.msg_csum(src[:n * L], L, mode=MODE)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    R = (L + 4095) // 4096
    hints = (0, R) if R > 1 else (0,)  # LAMPI_CSUM_ROWS_HINT: the fragment's rows as parallel row groups
    for tag, doff in (("aligned", 0), ("dst+8", 8)):
        descs = dv.make_copy_descs(src, offs, dst, offs + np.uint64(doff), np.full(n, L), np.full(n, L))
        for h in hints:
            dst[doff:doff + n * L].zero_()
            s = timed(lambda: dv.frag_bcopy_batch(descs, n=n, out=out, mode=MODE, rows_hint=h))
            ok = torch.equal(out, want) and torch.equal(dst[doff:doff + n * L], src[:n * L])
            print(f"bcopy L={L:8d} n={n:7d} {tag:8s} hint={h:4d} {2 * n * L / s / 8e12:.3f} of 8 TB/s  ok={ok}",
                  flush=True)
    # receive step: payloads at 72 + k * (72 + L + 8) with the expected checksum stamped at 64
    stride = 72 + L + 8
    m = min(n, (dst.numel() - 64) // stride)
    nic = dst[:m * stride]
    dv.msg_bcopy(src[:m * L], L, nic[72:], stride, out=out[:m], mode=MODE)
    nic.view(m, stride)[:, 64:68].copy_(out[:m].view(torch.uint8).view(m, 4))
    app = torch.zeros(m * L, dtype=torch.uint8, device="cuda")
    mo = np.arange(m, dtype=np.uint64)
    rd = dv.make_recv_descs(nic, mo * np.uint64(stride) + np.uint64(72), app, mo * np.uint64(L), np.full(m, L),
                            np.full(m, 1 << 40, dtype=np.int64))
    for h in hints:
        app.zero_()
        run = lambda: dv.copy_to_app_batch(rd, nic, expected_stride=stride, expected_offset=64, n=m,  # noqa: E731
                                           mode=MODE, rows_hint=h)
        s = timed(run)
        copied, csum, mask, nbad = run()
        ok = int(nbad.item()) == 0 and torch.equal(app, src[:m * L])
        print(f"recv  L={L:8d} n={m:7d}          hint={h:4d} {2 * m * L / s / 8e12:.3f} of 8 TB/s  ok={ok}", flush=True)
    del app
