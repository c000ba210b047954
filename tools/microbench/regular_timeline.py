"""Timeline of config B's kernel (crc_regular_kernel, read-only CRC of 4 KiB fragments in pairs) at 1 GiB and 16 GiB per
launch (diagnostic, never the product path): where a 1 GiB launch's extra ~15 us goes.

Runs lampi_diag_regular_timeline (launch_regular's grid and schedule; the kDiag instantiation stamps s_memrealtime,
100 MHz, per workgroup: entry, tables staged, each wave's exit, and the HW_ID / XCC_ID of its CU) after a warm-up of
the product path, checks the checksums against the product's, and prints: the span from the first entry to the last
exit against the rate of the middle of the launch; how long the start takes (until every resident slot has begun);
the tail (from the last workgroup's entry to the last exit) and how idle the CUs are in it; workgroup lifetimes.
Usage: python tools/microbench/regular_timeline.py [reps]
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from lampi_amd import _lib, device as dv  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
L = _lib.lib()
fn = L.lampi_diag_regular_timeline
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
stream = torch.cuda.current_stream()
buf = torch.empty(16 << 30, dtype=torch.uint8, device="cuda")
dv.fill_stream(buf, seed=2)
stamps = torch.zeros(16 * 45000, dtype=torch.int64, device="cuda")
for gib in (1, 4, 16):
    n = (gib << 30) // 4096
    src = buf[: n * 4096]
    want = dv.as_u32(dv.msg_csum(src, 4096, mode=dv.CRC32))
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    for _ in range(max(20, 320 // gib)):
        dv.msg_csum(src, 4096, mode=dv.CRC32, out=out)
    torch.cuda.synchronize()
    for r in range(reps):
        out.zero_()
        stamps.zero_()
        nwg = fn(src.data_ptr(), n, out.data_ptr(), stamps.data_ptr(), stream.cuda_stream)
        assert 0 < nwg <= 45000, nwg
        torch.cuda.synchronize()
        assert np.array_equal(dv.as_u32(out), want), "checksums"
        st = stamps[: 16 * nwg].view(nwg, 16).cpu().numpy()
        t0 = st[:, 0].min()
        ent = (st[:, 0] - t0) / 100.0  # us
        stg = (st[:, 1] - t0) / 100.0
        ext = (st[:, 2:6].max(axis=1) - t0) / 100.0
        span = ext.max()
        life = ext - ent
        # the CU: XCC_ID and HW_ID bits 8-15 (CU, SH, SE; bits 0-7 are the wave slot, SIMD and pipe)
        cu = ((st[:, 9].astype(np.int64) & 0xF) << 8) | ((st[:, 8].astype(np.int64) >> 8) & 0xFF)
        ucu = np.unique(cu)
        last_exit = np.array([ext[cu == c].max() for c in ucu])
        order = np.sort(ent)
        slots = min(nwg, 2 * ucu.size)
        start = order[slots - 1]  # every resident slot has begun
        # the steady rate: workgroups whose whole life lies in the middle 60% of the span
        mid = (ent > 0.2 * span) & (ext < 0.8 * span)
        done_mid = np.count_nonzero(mid)
        # HBM work done per us in the middle: count pairs of fragments by workgroups ending there
        ends = np.sort(ext)
        lo, hi = np.searchsorted(ends, 0.2 * span), np.searchsorted(ends, 0.8 * span)
        rate = (hi - lo) / (0.6 * span)  # workgroups finishing per us
        ideal = nwg / rate
        tail = span - ent.max()
        idle_tail = np.mean(span - last_exit)
        print(f"{gib:2d} GiB rep {r}: {nwg} workgroups on {ucu.size} CUs, span {span:8.1f} us, at the middle's rate "
              f"{ideal:8.1f} us (+{span - ideal:5.1f}); start {start:5.1f} us (first staging done "
              f"{np.sort(stg)[0]:4.1f}, median {np.median(stg - ent):4.1f} after entry); tail {tail:5.1f} us after the "
              f"last entry, CUs idle {idle_tail:5.1f} us on average before the end; lifetime median "
              f"{np.median(life):5.1f} us (p5 {np.percentile(life, 5):5.1f}, p95 {np.percentile(life, 95):5.1f}); "
              f"{done_mid} whole lives in the middle", flush=True)
