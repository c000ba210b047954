"""GPU parity of chained checksums over typemap pieces (lampi_chain_csum_batch).

The reference threads the CRC register / the partial-word sum state through one bcopy call per
typemap piece (src/path/gm/sendFrag.cc:157-217, src/path/common/BaseDesc.cc:72-163).  Pinned by
the reference's own chained results (tests/golden/fixtures.json `chain`: a message cut into
2-8 pieces, chained through the compiled MemFunctions.cc), then by the oracle on the packed
bytes (chained == contiguous is what the partial state guarantees) and by the oracle's
piece-by-piece chaining.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _dv():
    from lampi_amd import device as dv

    return dv


def _pieces_tensor(cuda, src, src_offs, dst, dst_offs, lens, partials=None):
    dv = _dv()
    return dv.make_copy_descs(src, src_offs, dst, dst_offs, lens, lens, partials)


def test_chain_reference_fixtures(cuda, oracle):
    """Every reference chain case as one batch; pieces also scattered to a gapped destination."""
    import torch

    dv = _dv()
    with open(os.path.join(os.path.dirname(__file__), "golden", "fixtures.json")) as f:
        cases = json.load(f)["chain"]
    msgs = [oracle.stream(c["seed"], c["off"], c["len"]) for c in cases]
    moff = np.concatenate([[0], np.cumsum([m.size + 16 for m in msgs])[:-1]]).astype(np.int64)
    src_host = np.zeros(int(moff[-1]) + msgs[-1].size + 16, np.uint8)
    for o, m in zip(moff, msgs):
        src_host[o:o + m.size] = m
    src = torch.from_numpy(src_host).to(cuda)
    so, do, ln, first = [], [], [], [0]
    dpos = 0
    for c, o in zip(cases, moff):
        bounds = [0] + c["cuts"] + [c["len"]]
        for a, b in zip(bounds, bounds[1:]):
            so.append(int(o) + a)
            do.append(dpos)
            ln.append(b - a)
            dpos += b - a + 5  # receive-side scatter: gaps between pieces
        first.append(len(so))
    dst = torch.zeros(dpos + 16, dtype=torch.uint8, device=cuda)
    pieces = _pieces_tensor(cuda, src, so, dst, do, ln)
    for mode, key in ((0, "crc"), (1, "sum")):
        got = dv.as_u32(dv.chain_csum_batch(pieces, first, mode=mode))
        want = np.array([c[key] for c in cases], np.uint32)
        assert np.array_equal(got, want), key
        whole = np.array([c[key + "_whole"] for c in cases], np.uint32)
        assert np.array_equal(got, whole)  # chained == contiguous (the reference's own identity)
    d = dst.cpu().numpy()
    for s_, d_, n_ in zip(so, do, ln):
        assert np.array_equal(d[d_:d_ + n_], src_host[s_:s_ + n_])


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_chain_random_gather(cuda, oracle, mode):
    """Send-side gather: scattered, misaligned pieces (1 B .. 20 KB, mostly small) packed into a
    contiguous payload per fragment."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(31 + mode)
    nfr = 400
    counts = rng.integers(0, 60, size=nfr)
    counts[::37] = 0
    lens = []
    for c in counts:
        small = rng.integers(1, 64, size=c)
        big = rng.integers(200, 20000, size=c)
        lens.append(np.where(rng.random(c) < 0.7, small, big))
    all_lens = np.concatenate(lens).astype(np.int64)
    npieces = all_lens.size
    src_bytes = 64 << 20
    src = torch.empty(src_bytes, dtype=torch.uint8, device=cuda)
    dv.fill_stream(src, seed=91)
    so = rng.integers(0, src_bytes - 20001, size=npieces)
    payload_len = np.array([int(x.sum()) for x in lens], np.int64)
    pay_off = np.concatenate([[0], np.cumsum(payload_len + 7)[:-1]])
    do, first = [], [0]
    for f in range(nfr):
        pos = pay_off[f]
        for ln in lens[f]:
            do.append(pos)
            pos += ln
        first.append(first[-1] + len(lens[f]))
    dst = torch.zeros(int(pay_off[-1] + payload_len[-1]) + 16, dtype=torch.uint8, device=cuda)
    parts = rng.integers(0, 2**32, size=npieces, dtype=np.uint64)
    pieces = _pieces_tensor(cuda, src, so, dst, do, all_lens, parts)
    got = dv.as_u32(dv.chain_csum_batch(pieces, first, mode=mode))
    host_src = src.cpu().numpy()
    packed = dst.cpu().numpy()
    pos = 0
    for f in range(nfr):
        for k in range(first[f], first[f + 1]):
            assert np.array_equal(packed[do[k]:do[k] + all_lens[k]], host_src[so[k]:so[k] + all_lens[k]])
    fparts = np.array([parts[first[f]] if first[f + 1] > first[f] else 0xFFFFFFFF for f in range(nfr)], np.uint64)
    want = oracle.desc_batch(packed, pay_off.astype(np.uint64), payload_len.astype(np.uint32),
                             fparts.astype(np.uint32) if mode == 0 else None, mode)
    assert np.array_equal(got, want)
    # piece-by-piece chaining through the oracle, as the reference's send loop does it
    for f in rng.choice(nfr, size=12, replace=False):
        crc, tot, pi, pl = int(fparts[f]), 0, 0, 0
        for k in range(first[f], first[f + 1]):
            piece = host_src[so[k]:so[k] + all_lens[k]]
            crc = oracle.uicrc(piece, piece.size, crc)
            s, pi, pl = oracle.uicsum(piece, piece.size, pi, pl)
            tot = (tot + s) & 0xFFFFFFFF
        assert got[f] == (crc if mode == 0 else tot)


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_chain_strided_vector(cuda, oracle, mode):
    """A vector datatype: 8000 blocks of 8 bytes, stride 24 (one fragment of tiny pieces)."""
    import torch

    dv = _dv()
    n, blk, stride = 8000, 8, 24
    src = torch.empty(n * stride + 64, dtype=torch.uint8, device=cuda)
    dv.fill_stream(src, seed=92)
    dst = torch.zeros(n * blk, dtype=torch.uint8, device=cuda)
    so = 3 + np.arange(n) * stride
    do = np.arange(n) * blk
    pieces = _pieces_tensor(cuda, src, so, dst, do, np.full(n, blk))
    got = dv.as_u32(dv.chain_csum_batch(pieces, [0, n], mode=mode))
    packed = dst.cpu().numpy()
    h = src.cpu().numpy()
    assert np.array_equal(packed, np.concatenate([h[o:o + blk] for o in so]))
    want = oracle.uicrc(packed) if mode == 0 else oracle.uicsum(packed)[0]
    assert got[0] == want


def test_chain_empty_and_zero_length(cuda):
    import torch

    dv = _dv()
    src = torch.arange(64, dtype=torch.int32, device=cuda).to(torch.uint8)
    dst = torch.zeros(64, dtype=torch.uint8, device=cuda)
    pieces = _pieces_tensor(cuda, src, [0, 5, 9], dst, [0, 0, 0], [0, 0, 0])
    for mode, empty in ((0, 0xFFFFFFFF), (1, 0)):
        got = dv.as_u32(dv.chain_csum_batch(pieces, [0, 0, 3, 3], mode=mode))
        assert got[0] == empty and got[2] == empty
        assert got[1] == (0xFFFFFFFF if mode == 0 else 0)  # three empty pieces: the register passes through


@pytest.mark.parametrize("mode", [0, 1, 2], ids=["crc", "sum", "off"])
def test_chain_copy_to_app_verdicts(cuda, oracle, mode):
    """CopyToApp's non-contiguous branch (lampi_chain_copy_to_app_batch; ref src/path/common/BaseDesc.cc:326-340,
    non_contiguous_copy :72-163, CheckData src/path/gm/recvFrag.h:213-257): the reference's 150 chain fixtures
    as received fragments scattered into typemap pieces of an application buffer, plus fragments with no
    pieces (AppBufferLen <= 0) and with zero-length pieces.  ~30% of the expected checksums are corrupted
    (dataChecksum |= 0xA4A4, recvFrag.h:215-229); the pieces' partial is garbage (the batch starts CRC from
    CRC_INITIAL_REGISTER).  copied / csum / mask / nbad against oracle.non_contiguous_copy_to_app, the delivered
    bytes against the fragments."""
    import torch

    from oracle.oracle import non_contiguous_copy_to_app

    dv = _dv()
    rng = np.random.default_rng(404 + mode)
    with open(os.path.join(os.path.dirname(__file__), "golden", "fixtures.json")) as f:
        cases = json.load(f)["chain"]
    msgs = [oracle.stream(c["seed"], c["off"], c["len"]) for c in cases]
    # a few extra received fragments: no pieces at all, and zero-length pieces around real ones
    msgs += [np.zeros(0, np.uint8), np.zeros(0, np.uint8), oracle.stream(9, 0, 300)]
    cuts = [c["cuts"] for c in cases] + [None, [], [0, 0, 150, 150, 300]]
    moff = np.concatenate([[0], np.cumsum([m.size + 16 for m in msgs])[:-1]]).astype(np.int64)
    src_host = np.zeros(int(moff[-1]) + msgs[-1].size + 16, np.uint8)
    for o, m in zip(moff, msgs):
        src_host[o:o + m.size] = m
    src = torch.from_numpy(src_host).to(cuda)
    so, do, ln, first, want, exp = [], [], [], [0], [], []
    dpos = 0
    for m, o, cu in zip(msgs, moff, cuts):
        parts = []
        if cu is not None:
            bounds = [0] + list(cu) + [m.size]
            for a, b in zip(bounds, bounds[1:]):
                so.append(int(o) + a)
                do.append(dpos)
                ln.append(b - a)
                parts.append(m[a:b])
                dpos += b - a + int(rng.integers(1, 9))  # the typemap's holes in the application buffer
        first.append(len(so))
        true = non_contiguous_copy_to_app(oracle, parts, 0, mode)[1]
        e = true | 0xA4A4 if rng.random() < 0.3 else true
        exp.append(e)
        want.append(non_contiguous_copy_to_app(oracle, parts, e, mode))
    dst = torch.full((dpos + 16,), 0x5C, dtype=torch.uint8, device=cuda)
    partials = rng.integers(0, 1 << 32, size=len(so), dtype=np.uint64)
    pieces = dv.make_copy_descs(src, so, dst, do, ln, ln, partials)
    expected = torch.from_numpy(np.array(exp, np.uint32).view(np.int32)).to(cuda)
    copied, csum, mask, nbad = dv.chain_copy_to_app_batch(pieces, first, None if mode == 2 else expected, 4, mode=mode)
    nf = len(msgs)
    want_copied = np.array([w[0] for w in want], np.int64)
    want_csum = np.array([w[1] for w in want], np.uint32)
    assert np.array_equal(copied.cpu().numpy(), want_copied), np.nonzero(copied.cpu().numpy() != want_copied)[0][:8]
    assert np.array_equal(dv.as_u32(csum), want_csum)
    bad = want_copied == -1
    assert np.array_equal(dv.mask_bits(mask, nf), bad)
    assert int(nbad.item()) == int(bad.sum())
    assert (bad.any() and not bad.all()) if mode != 2 else not bad.any()
    want_dst = np.full(dpos + 16, 0x5C, np.uint8)
    for s_, d_, n_ in zip(so, do, ln):
        want_dst[d_:d_ + n_] = src_host[s_:s_ + n_]
    assert np.array_equal(dst.cpu().numpy(), want_dst)  # delivered whatever the verdict, holes untouched
