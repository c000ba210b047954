"""Timeline of the read-only CRC piece-stream kernel on config C (diagnostic, never the product path).

Runs lampi_diag_stream_timeline (the product grid and schedule; the kDiag instantiation of
crc_stream_kernel stamps s_memrealtime, 100 MHz, per workgroup: entry, set-up done, first row checksummed,
rows done, exit) after a warm-up of the product path, checks the batch digest, and prints where a
workgroup's life goes and how many workgroups are resident over the kernel's span.
Usage: python tools/microbench/stream_timeline.py [reps]
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from lampi_amd import _lib, device as dv, shard  # noqa: E402
from lampi_amd.workload import zipf_lengths  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
lens = zipf_lengths(4 << 30)
offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
total = int(lens.sum(dtype=np.uint64))
buf = torch.empty(total, dtype=torch.uint8, device="cuda")
dv.fill_stream(buf, seed=5)
descs = dv.make_descs(buf, offs, lens)
out = torch.empty(lens.size, dtype=torch.int32, device="cuda")
for _ in range(400):
    dv.frag_csum_batch(descs, mode=dv.CRC32, out=out)
torch.cuda.synchronize()
L = _lib.lib()
fn = L.lampi_diag_stream_timeline
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
stamps = torch.zeros(16 * 8192, dtype=torch.int64, device="cuda")
stream = torch.cuda.current_stream()
with open(os.path.join(ROOT, "tests", "golden", "fixtures.json")) as f:
    gold = json.load(f)["digests"]["C"]
res = []
for r in range(reps):
    out.zero_()
    nwg = fn(descs.data_ptr(), lens.size, out.data_ptr(), stamps.data_ptr(), stream.cuda_stream)
    assert nwg > 0 and nwg <= 8192, nwg
    torch.cuda.synchronize()
    got = shard.digest(dv.as_u32(out), np.arange(lens.size, dtype=np.uint64))
    assert got == (gold["crc_xor"], gold["crc_wsum"]), "digest"
    st = stamps[: 16 * nwg].view(nwg, 16).cpu().numpy()
    t = st[:, [0, 1, 2, 3, 4, 7, 8, 9]].astype(np.float64) * 10.0 / 1000.0  # us (100 MHz)
    t -= t[:, 0].min()
    tab = t[:, 5] - t[:, 0]   # entry -> descriptors and tables in
    scan = t[:, 6] - t[:, 5]  # -> prefix scan done
    chs = t[:, 1] - t[:, 6]   # -> chains set up
    rlat = t[:, 7] - t[:, 1]  # -> first rows arrived
    span = t[:, 4].max()
    life = t[:, 4] - t[:, 0]
    pro = t[:, 1] - t[:, 0]
    first = t[:, 2] - t[:, 1]
    body = t[:, 3] - t[:, 2]
    epi = t[:, 4] - t[:, 3]
    # resident workgroups over time (1 us bins)
    nb = int(span) + 1
    occ = np.zeros(nb)
    for a, b in zip(t[:, 0], t[:, 4]):
        occ[int(a):int(b) + 1] += 1
    res.append(span)
    print(f"rep {r}: {nwg} workgroups, span {span:.1f} us ({total / span / 1e6 / 8:.1%} of 8 TB/s), "
          f"life mean {life.mean():.1f} us | entry->desc+tables {tab.mean():.2f} scan {scan.mean():.2f} chains {chs.mean():.2f} "
          f"first-row latency {rlat.mean():.2f} | entry->set-up {pro.mean():.2f} | set-up->first row {first.mean():.2f} "
          f"| rows {body.mean():.1f} | join+store {epi.mean():.2f} | resident mean {occ[:-1].mean():.0f} "
          f"first-10us {occ[:10].mean():.0f} last-20us {occ[-21:-1].mean():.0f} last-50us {occ[-51:-1].mean():.0f}",
          flush=True)
    if r == reps - 1:
        hw = st[:, 5].astype(np.int64)
        xcc = st[:, 6].astype(np.int64) & 0xF
        print("start-time deciles (us):", np.percentile(t[:, 0], [10, 50, 90, 99, 100]).round(1).tolist())
        print("exit-time of the last 1% (us):", np.sort(t[:, 4])[-max(1, nwg // 100):][[0, -1]].round(1).tolist())
        print("life deciles (us):", np.percentile(life, [10, 50, 90, 100]).round(1).tolist())
        print("xcc ids seen:", sorted(set(xcc.tolist()))[:16], "hw_id sample:", [hex(x) for x in hw[:4]])
        np.save(os.path.join(ROOT, "gpurun_out", "stream_timeline.npy"), st)
