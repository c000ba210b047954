"""GPU parity of the 64-bit additive checksum (csum / bcopy_csum).

Host entry points (computed on the GPU) against the reference's own results
(tests/golden/csum64.json, from the compiled MemFunctions.cc), and the device batch
(lampi_frag_csum64_batch) against the oracle's restatement.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "csum64.json")


def test_host_csum64_reference_fixtures(cuda):
    import lampi_amd as la
    from oracle.oracle import splitmix_stream

    with open(GOLD) as f:
        g = json.load(f)
    for c in g["single"]:
        st = la.PartialState64(c["plong"], c["plen"])
        got = la.csum(splitmix_stream(c["seed"], c["off"], c["len"]), c["len"], st)
        assert (got, st.plong, st.plen) == (c["sum"], c["plong_out"], c["plen_out"]), c["len"]
    for c in g["chain"]:
        buf = splitmix_stream(c["seed"], c["off"], c["len"])
        bounds = [0] + c["cuts"] + [c["len"]]
        st, tot = la.PartialState64(), 0
        for a, b in zip(bounds, bounds[1:]):
            tot = (tot + la.csum(buf[a:b], b - a, st)) % 2**64
        assert tot == c["sum"]
    for c in g["bcopy"]:
        total = max(c["copylen"], c["clen"])
        src = np.zeros(total + 16, np.uint8)
        src[c["src_align"]:c["src_align"] + total] = splitmix_stream(c["seed"], c["off"], total)
        dst = np.zeros(total + 16, np.uint8)
        st = la.PartialState64(c["plong"], c["plen"])
        got = la.bcopy_csum(src[c["src_align"]:c["src_align"] + total], dst[c["dst_align"]:], c["copylen"], c["clen"],
                            st)
        assert (got, st.plong, st.plen) == (c["sum"], c["plong_out"], c["plen_out"])
        assert np.array_equal(dst[c["dst_align"]:c["dst_align"] + c["copylen"]],
                              src[c["src_align"]:c["src_align"] + c["copylen"]])


def test_host_csum64_large(cuda, oracle):
    """Multi-piece host path (several MiB, every start phase)."""
    import lampi_amd as la

    rng = np.random.default_rng(64)
    data = rng.integers(0, 256, size=(9 << 20) + 13, dtype=np.uint8)
    for n in [(9 << 20) + 13, (1 << 20) + 7, 4096 * 17]:
        for plen in range(8):
            plong = int(rng.integers(0, 2**63)) & ((1 << (8 * plen)) - 1)
            st = la.PartialState64(plong, plen)
            got = la.csum(data[:n], n, st)
            assert (got, st.plong, st.plen) == oracle.csum(data[:n], n, plong, plen), (n, plen)


def test_device_csum64_batch(cuda, oracle):
    import torch

    from lampi_amd import device as dv

    rng = np.random.default_rng(65)
    base = torch.empty(32 << 20, dtype=torch.uint8, device=cuda)
    dv.fill_stream(base, seed=66)
    host = base.cpu().numpy()
    lens = np.concatenate([np.repeat([0, 1, 7, 8, 9, 63, 64, 4095, 4096, 4097, 65456], 16),
                           rng.integers(0, 70000, size=3000)]).astype(np.uint64)
    offs = (rng.integers(0, (32 << 20) - 70000, size=lens.size) // 16 * 16 +
            np.tile(np.arange(16), lens.size // 16 + 1)[:lens.size]).astype(np.uint64)
    descs = dv.make_descs(base, offs, lens)
    got = dv.frag_csum64_batch(descs).cpu().numpy().view(np.uint64)
    want = np.array([oracle.csum(host[int(o):int(o) + int(n)], int(n))[0] for o, n in zip(offs, lens)], np.uint64)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(lens[i]), int(offs[i]) % 16) for i in bad[:8]]
