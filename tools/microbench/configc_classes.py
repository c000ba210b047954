#!/usr/bin/env python3
"""Config C by size class on the current product (round 6): the whole batch and each class alone --
one-row fragments (<= 4 KiB), 2-7 rows, 8-16 rows -- as descriptor batches over the same 4 GiB buffer (each class keeps
its fragments' own addresses), read-only CRC and SUM; % of the 8 TB/s roofline by HIP events over 20 calls after a
0.3 s warm-up, the checksums of every class compared with the whole batch's."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from lampi_amd import device as dv  # noqa: E402
from lampi_amd.workload import zipf_lengths  # noqa: E402


def timed(descs, n, mode, out):
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < 0.3 or k < 10:
        dv.frag_csum_batch(descs, n=n, mode=mode, out=out)
        k += 1
        if k % 50 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(20):
        dv.frag_csum_batch(descs, n=n, mode=mode, out=out)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 20 / 1e3


def main():
    lens = zipf_lengths(4 << 30)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.sum(dtype=np.uint64))
    buf = torch.empty(total, dtype=torch.uint8, device="cuda")
    dv.fill_stream(buf, seed=5)
    rows = (lens.astype(np.int64) + 4095) // 4096
    classes = {"all": np.ones(lens.size, bool), "1 row (<= 4 KiB)": rows == 1, "2-7 rows": (rows >= 2) & (rows <= 7),
               "8-16 rows": rows >= 8, "2-16 rows": rows >= 2}
    for mode, name in ((dv.CRC32, "crc"), (dv.SUM32, "sum")):
        whole = None
        for cname, m in classes.items():
            idx = np.nonzero(m)[0]
            descs = dv.make_descs(buf, offs[idx], lens[idx])
            out = torch.empty(idx.size, dtype=torch.int32, device="cuda")
            sec = timed(descs, idx.size, mode, out)
            got = dv.as_u32(out)
            if cname == "all":
                whole = got
                ok = True
            else:
                ok = bool(np.array_equal(got, whole[idx]))
            b = int(lens[idx].sum(dtype=np.uint64))
            print(f"{name} {cname:18s} fragments {idx.size:7d} bytes {b:11d} {sec * 1e6:8.1f} us "
                  f"{b / sec / 8e12 * 100:5.1f}% same {ok}", flush=True)


if __name__ == "__main__":
    main()
