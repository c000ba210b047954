"""Probe: small fragments (pack path) mixed with other fragments in one wave, vs the oracle."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from lampi_amd import device as dv  # noqa: E402
from oracle.oracle import Restatement  # noqa: E402

ref = Restatement()
base = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
dv.fill_stream(base, seed=5)
host = base.cpu().numpy()
cases = {
    "pack+row": ([4096, 16384], [64, 5000]),
    "row+pack": ([4096, 16384], [5000, 64]),
    "pack+small": ([4096, 8193], [64, 100]),
    "small+pack": ([8193, 4096], [100, 64]),
    "pack+row1k": ([4096, 16384], [64, 1000]),
    "edges64": ([65536 + 64 * 0 + a for a in range(17)], [64] * 17),
    "pack2+row": ([4096, 8192, 16384], [64, 64, 5000]),
}
for name, (offs, lens) in cases.items():
    offs = np.array(offs, np.uint64)
    lens = np.array(lens, np.uint64)
    parts = np.full(offs.size, 0xFFFFFFFF, np.uint64)
    got = dv.as_u32(dv.frag_csum_batch(dv.make_descs(base, offs, lens, parts), mode=dv.CRC32))
    want = ref.desc_batch(host, offs, lens, parts.astype(np.uint32), 0)
    print(name, "ok" if np.array_equal(got, want) else
          f"BAD got {[hex(x) for x in got]} want {[hex(x) for x in want]}")
