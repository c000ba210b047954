"""Descriptor batches of large uniform fragments through the piece streams (lampi_frag_csum_batch):
few fragments per workgroup, so every fragment spans several chains and stream_join decides.
python tools/microbench/bigdesc_scan.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lampi_amd import device as dv  # noqa: E402

buf = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
dv.fill_stream(buf, seed=9)
for L in (65536, 262144, 1 << 20, 4 << 20):
    n = (1 << 30) // L
    d = dv.make_descs(buf, np.arange(n, dtype=np.uint64) * np.uint64(L), np.full(n, L, np.uint64))
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    for _ in range(20):
        dv.frag_csum_batch(d, n=n, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        dv.frag_csum_batch(d, n=n, out=out)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 20 / 1e3
    print(f"descriptors L={L:8d} n={n:6d} 1 GiB crc {n * L / t / 8e12:.3f} of 8 TB/s", flush=True)
