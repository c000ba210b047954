"""Per-kernel device time of tiny launches, replayed from HIP graphs of 8 nodes (no host
overhead): a one-element torch add (the launch floor) against lampi_frag_csum_batch and
lampi_msg_csum on one 4 KiB fragment.  python tools/microbench/launch_floor.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lampi_amd import device as dv  # noqa: E402


def graph_us(fn, nodes=8, reps=200):
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(nodes):
            fn()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * nodes) * 1e3


x = torch.zeros(1, device="cuda")
buf = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
dv.fill_stream(buf, seed=1)
out = torch.empty(256, dtype=torch.int32, device="cuda")
print(f"one-element add            {graph_us(lambda: x.add_(1)):6.2f} us per kernel", flush=True)
for n in (1, 16, 256):
    d = dv.make_descs(buf, np.arange(n, dtype=np.uint64) * 4096, np.full(n, 4096, np.uint64))
    print(f"frag_csum_batch n={n:<4d}     {graph_us(lambda: dv.frag_csum_batch(d, n=n, out=out)):6.2f} us per call",
          flush=True)
    print(f"frag_csum_batch sum n={n:<4d} {graph_us(lambda: dv.frag_csum_batch(d, n=n, out=out, mode=dv.SUM32)):6.2f} us per call",
          flush=True)
    print(f"msg_csum n={n:<4d}            {graph_us(lambda: dv.msg_csum(buf, 4096, out=out, msg_len=n * 4096)):6.2f} us per call",
          flush=True)
