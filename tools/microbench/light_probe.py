"""One shape per run for counter collection: lampi_msg_bcopy CRC of 1M x 4 KiB into a packed
destination (the table-light copy), or with --gm 16,384 x 65,456 B into 64 KiB slots at +72.
python tools/microbench/light_probe.py [--gm] [--reps N]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

from lampi_amd import device as dv  # noqa: E402

gm = "--gm" in sys.argv
reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 5
L, n, stride, off = (65456, 1 << 14, 65536, 72) if gm else (4096, 1 << 20, 4096, 0)
msg = torch.empty(n * L, dtype=torch.uint8, device="cuda")
dv.fill_stream(msg, seed=13)
dst = torch.zeros(off + n * stride, dtype=torch.uint8, device="cuda")
out = torch.empty(n, dtype=torch.int32, device="cuda")
for _ in range(reps):
    dv.msg_bcopy(msg, L, dst[off:], stride, mode=dv.CRC32, out=out)
torch.cuda.synchronize()
print("ok", torch.equal(out, dv.msg_csum(msg, L)))
