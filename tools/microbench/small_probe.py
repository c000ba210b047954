import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
from lampi_amd import device as dv
buf = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
dv.fill_stream(buf, seed=9)
for n in (1, 4096):
    d = dv.make_descs(buf, np.arange(n, dtype=np.uint64) * np.uint64(4096), np.full(n, 4096, np.uint64))
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    for _ in range(30):
        dv.frag_csum_batch(d, n=n, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        dv.frag_csum_batch(d, n=n, out=out)
    torch.cuda.synchronize()
    print(n, (time.perf_counter() - t0) / 50 * 1e6, "us/call host", flush=True)
