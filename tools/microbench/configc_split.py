"""Where config C's time goes: the piece-stream kernel (lampi_frag_csum_batch) on the whole Zipf
batch and on its size classes alone (fragments < 4 KiB / >= 4 KiB, and < 1 KiB / >= 16 KiB),
same buffer and descriptors.  Prints each subset's bytes, kernel time and fraction of 8 TB/s.

python tools/microbench/configc_split.py [--quick]   (--quick: the whole batch and the prologue only)
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lampi_amd import device as dv  # noqa: E402
from lampi_amd.workload import zipf_lengths  # noqa: E402

lens = zipf_lengths(4 << 30)
offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
total = int(lens.sum(dtype=np.uint64))
buf = torch.empty(total, dtype=torch.uint8, device="cuda")
dv.fill_stream(buf, seed=5)


def timed(descs, n, reps=30):
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    for _ in range(200):
        dv.frag_csum_batch(descs, n=n, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        dv.frag_csum_batch(descs, n=n, out=out)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


QUICK = "--quick" in sys.argv
for name, sel in (("all", np.ones(lens.size, bool)),) + (() if QUICK else (
        ("<4KiB", lens < 4096), (">=4KiB", lens >= 4096), ("<1KiB", lens < 1024), (">=16KiB", lens >= 16384))):
    idx = np.nonzero(sel)[0]
    d = dv.make_descs(buf, offs[idx], lens[idx])
    b = int(lens[idx].sum(dtype=np.uint64))
    t = timed(d, idx.size)
    print(f"{name:8s} {idx.size:7d} fragments {b / 2**30:6.3f} GiB  {t * 1e3:7.3f} ms  "
          f"{b / t / 8e12:.3f} of 8 TB/s", flush=True)

if QUICK:
    zl = np.zeros(lens.size, dtype=lens.dtype)
    t = timed(dv.make_descs(buf, offs, zl), lens.size)
    print(f"empty fragments: {t * 1e3:7.3f} ms", flush=True)
    sys.exit(0)

# the two size classes at once, on two streams (the small fragments' latency-bound work
# overlapping the large fragments' streaming)
big = np.nonzero(lens >= 4096)[0]
small = np.nonzero(lens < 4096)[0]
db = dv.make_descs(buf, offs[big], lens[big])
ds = dv.make_descs(buf, offs[small], lens[small])
ob = torch.empty(big.size, dtype=torch.int32, device="cuda")
os_ = torch.empty(small.size, dtype=torch.int32, device="cuda")
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
main = torch.cuda.current_stream()


def both():
    ev = torch.cuda.Event()
    ev.record(main)
    sa.wait_event(ev)
    sb.wait_event(ev)
    dv.frag_csum_batch(db, n=big.size, out=ob, stream=sa)
    dv.frag_csum_batch(ds, n=small.size, out=os_, stream=sb)
    ea, eb = torch.cuda.Event(), torch.cuda.Event()
    ea.record(sa)
    eb.record(sb)
    main.wait_event(ea)
    main.wait_event(eb)


for _ in range(200):
    both()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(main)
for _ in range(30):
    both()
e1.record(main)
torch.cuda.synchronize()
t = e0.elapsed_time(e1) / 30 / 1e3
print(f"two streams: >=4KiB || <4KiB  {t * 1e3:7.3f} ms  {total / t / 8e12:.3f} of 8 TB/s", flush=True)

# workgroup prologue: the same number of fragments (and workgroups), every fragment empty / 64 B
zl = np.zeros(lens.size, dtype=lens.dtype)
t = timed(dv.make_descs(buf, offs, zl), lens.size)
print(f"empty fragments ({lens.size} -> {(lens.size + 95) // 96} workgroups): {t * 1e3:7.3f} ms", flush=True)
t = timed(dv.make_descs(buf, offs, zl + 64), lens.size)
print(f"64-byte fragments: {t * 1e3:7.3f} ms", flush=True)

# bytes per 96-fragment workgroup in the product's order
g = np.add.reduceat(lens.astype(np.int64), np.arange(0, lens.size, 96))
print(f"workgroup bytes: mean {g.mean() / 1024:.0f} KiB, max {g.max() / 1024:.0f} KiB, "
      f"p99 {np.percentile(g, 99) / 1024:.0f} KiB, last 512 mean {g[-512:].mean() / 1024:.0f} KiB", flush=True)

# the same fragments dealt into byte-balanced workgroups (sorted by length, snake order): no
# locality between the fragments of a workgroup, equal bytes per workgroup
order = np.argsort(-lens, kind="stable")
ng = (lens.size + 95) // 96
slot = np.arange(lens.size)
rnd, pos = slot // ng, slot % ng
grp = np.where(rnd % 2 == 0, pos, ng - 1 - pos)
perm = order[np.lexsort((rnd, grp))]
gb = np.add.reduceat(lens[perm].astype(np.int64), np.arange(0, lens.size, 96))
t = timed(dv.make_descs(buf, offs[perm], lens[perm]), lens.size)
print(f"balanced order (workgroup bytes max/mean {gb.max() / gb.mean():.2f}): {t * 1e3:7.3f} ms  "
      f"{total / t / 8e12:.3f} of 8 TB/s", flush=True)
# a random order (no locality, unbalanced) to separate the two effects
rp = np.random.default_rng(7).permutation(lens.size)
t = timed(dv.make_descs(buf, offs[rp], lens[rp]), lens.size)
print(f"random order: {t * 1e3:7.3f} ms  {total / t / 8e12:.3f} of 8 TB/s", flush=True)
