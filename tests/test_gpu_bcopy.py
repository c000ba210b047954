"""GPU parity of the fused copy + checksum batch (lampi_frag_bcopy_batch).

bcopy_uicrc / bcopy_uicsum (ref src/util/MemFunctions.cc:1263-1321, 518-875) copy `copylen`
bytes and checksum max(copylen, csumlen) bytes; the residue is checksummed, never copied.
Checked bit-exact: checksums against the reference-generated fixtures (tests/golden, `bcopy`)
and the oracle; destination bytes against the source, with every byte outside the copies
left untouched (sentinel stream).
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EDGE_LENS = [0, 1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 63, 64, 65, 127, 1023, 1024, 1025, 1976, 2031, 2047, 2048, 2049,
             4092, 4095, 4096, 4097, 4098, 4099, 4111, 4113, 8191, 8192, 8193, 8194, 12289, 16384, 16385, 65455,
             65456]
# (16-2048: the CRC copy's half frame -- 2 KiB, two chunks per lane; 2049 the first full-frame length)
# (4097-4099, 8193, 8194, 12289: a 4 KiB frame's padding leaves the fragment's first bytes -- and the
# register injected there -- in the last chunk of a row, spilling into the next row's first chunk)


def _dv():
    from lampi_amd import device as dv

    return dv


def _layout(totals, copylens, src_align, dst_align):
    """Disjoint 64-byte-aligned slots (plus 64 bytes of gap) for every source and destination."""
    slot_s = (np.asarray(totals, np.int64) + 16 + 64 + 63) // 64 * 64
    slot_d = (np.asarray(copylens, np.int64) + 16 + 64 + 63) // 64 * 64
    so = np.concatenate([[0], np.cumsum(slot_s)[:-1]]) + np.asarray(src_align, np.int64)
    do = np.concatenate([[0], np.cumsum(slot_d)[:-1]]) + np.asarray(dst_align, np.int64)
    return so.astype(np.uint64), do.astype(np.uint64), int(slot_s.sum()), int(slot_d.sum())


def _run(cuda, oracle, copylens, csumlens, src_align, dst_align, partials, mode, src_fill=None, rows_hint=0):
    """Run one batch; return (checksums, expected checksums, dst bytes, expected dst bytes)."""
    import torch

    dv = _dv()
    cl = np.asarray(copylens, np.uint64)
    sl = np.asarray(csumlens, np.uint64)
    tot = np.maximum(cl, sl)
    so, do, ns, nd = _layout(tot, cl, src_align, dst_align)
    src = torch.empty(max(ns, 64), dtype=torch.uint8, device=cuda)
    dv.fill_stream(src, seed=41)
    host_src = src.cpu().numpy()
    if src_fill is not None:  # caller-provided payloads (fixture slices)
        for i, b in enumerate(src_fill):
            host_src[int(so[i]):int(so[i]) + b.size] = b
        src.copy_(torch.from_numpy(host_src).to(cuda))
    dst = torch.empty(max(nd, 64), dtype=torch.uint8, device=cuda)
    dv.fill_stream(dst, seed=42)
    want_dst = dst.cpu().numpy().copy()
    for i in range(cl.size):
        a, b, n = int(so[i]), int(do[i]), int(cl[i])
        want_dst[b:b + n] = host_src[a:a + n]
    descs = dv.make_copy_descs(src, so, dst, do, cl, sl, partials)
    got = dv.as_u32(dv.frag_bcopy_batch(descs, mode=mode, rows_hint=rows_hint))
    want = oracle.desc_batch(host_src, so, tot.astype(np.uint32),
                             None if mode == 1 else np.asarray(partials, np.uint64).astype(np.uint32), mode)
    return got, want, dst.cpu().numpy(), want_dst


def _assert_same(got, want, dgot, dwant, info):
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [info(i) for i in bad[:8]]
    diff = np.nonzero(dgot != dwant)[0]
    assert diff.size == 0, f"{diff.size} destination bytes differ, first at {int(diff[0])}"


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_bcopy_batch_reference_fixtures(cuda, oracle, mode):
    """The reference's own bcopy_uicrc / bcopy_uicsum results (tests/golden/fixtures.json)."""
    with open(os.path.join(os.path.dirname(__file__), "golden", "fixtures.json")) as f:
        cases = json.load(f)["bcopy"]
    if mode == 1:  # the batch starts every fragment from a fresh partial-word state
        cases = [c for c in cases if c["plen"] == 0]
    cl = [c["copylen"] for c in cases]
    sl = [c["clen"] for c in cases]
    payload = [oracle.stream(c["seed"], c["off"], max(c["copylen"], c["clen"])) for c in cases]
    got, want, dgot, dwant = _run(cuda, oracle, cl, sl, [c["src_align"] for c in cases],
                                  [c["dst_align"] for c in cases], [c["partial"] for c in cases], mode, payload)
    fx = np.array([c["crc"] if mode == 0 else c["sum"] for c in cases], np.uint32)
    assert np.array_equal(want, fx)  # oracle == reference on these inputs
    _assert_same(got, fx, dgot, dwant, lambda i: (cl[i], sl[i], cases[i]["src_align"], cases[i]["dst_align"]))


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_bcopy_batch_edges_and_alignment(cuda, oracle, mode):
    """Every edge length x source/destination misalignment x (copy =, <, > checksum length)."""
    rng = np.random.default_rng(515)
    cl, sl, sa, da = [], [], [], []
    for L in EDGE_LENS:
        for a in range(16):
            for kind in range(3):
                b = int(rng.integers(0, 16))
                short = int(rng.integers(0, L + 1))
                cl.append(L if kind != 1 else short)  # kind 1: copylen < csumlen (receive side)
                sl.append(L if kind != 2 else short)  # kind 2: csumlen < copylen
                sa.append(a)
                da.append(b)
    parts = rng.integers(0, 2**32, size=len(cl), dtype=np.uint64)
    parts[::4] = 0xFFFFFFFF
    got, want, dgot, dwant = _run(cuda, oracle, cl, sl, sa, da, parts, mode)
    _assert_same(got, want, dgot, dwant, lambda i: (cl[i], sl[i], sa[i], da[i]))


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
@pytest.mark.parametrize("rows_hint", [2, 3, 16, 64])
def test_bcopy_batch_row_groups(cuda, oracle, rows_hint, mode):
    """LAMPI_CSUM_ROWS_HINT: each fragment's rows run as row groups (ceil(R / hint) rows each) in
    parallel and are joined afterwards (CRC: shifted and XORed; SUM: added) -- edge lengths x
    alignments x copy =, <, > checksum length, then fragments of up to ~300 KB (more rows than the
    hint: groups of several rows, a short last group), every checksum and destination byte against
    the oracle."""
    rng = np.random.default_rng(900 + rows_hint)
    cl, sl, sa, da = [], [], [], []
    for L in EDGE_LENS:
        for a in range(0, 16, 5):
            for kind in range(3):
                short = int(rng.integers(0, L + 1))
                cl.append(L if kind != 1 else short)
                sl.append(L if kind != 2 else short)
                sa.append(a)
                da.append(int(rng.integers(0, 16)))
    n = 600
    big_c = rng.integers(0, 300000, size=n)
    big_s = np.where(rng.random(n) < 0.3, rng.integers(0, 300000, size=n), big_c)
    cl += big_c.tolist()
    sl += big_s.tolist()
    sa += rng.integers(0, 16, size=n).tolist()
    da += rng.integers(0, 16, size=n).tolist()
    parts = rng.integers(0, 2**32, size=len(cl), dtype=np.uint64)
    got, want, dgot, dwant = _run(cuda, oracle, cl, sl, sa, da, parts, mode, rows_hint=rows_hint)
    _assert_same(got, want, dgot, dwant, lambda i: (cl[i], sl[i], sa[i], da[i]))


def test_bcopy_batch_random(cuda, oracle):
    rng = np.random.default_rng(77)
    n = 6000
    cl = rng.integers(0, 70000, size=n)
    sl = np.where(rng.random(n) < 0.3, rng.integers(0, 70000, size=n), cl)
    sa = rng.integers(0, 16, size=n)
    da = np.where(rng.random(n) < 0.5, sa, rng.integers(0, 16, size=n))
    parts = rng.integers(0, 2**32, size=n, dtype=np.uint64)
    for mode in (0, 1):
        got, want, dgot, dwant = _run(cuda, oracle, cl, sl, sa, da, parts, mode)
        _assert_same(got, want, dgot, dwant, lambda i: (int(cl[i]), int(sl[i]), int(sa[i]), int(da[i])))


@pytest.mark.parametrize("n,layout", [(40, "aligned"), (40, "src8"), (3000, "mixed"), (30000, "mixed"),
                                      (30000, "src8")])
def test_bcopy_batch_sum_streams(cuda, oracle, n, layout):
    """SUM fused copies of descriptor batches (sum_copy_wg_kernel: one workgroup per fragment,
    unaligned 16-byte loads and stores, the last 1-15 bytes and the chunk a short copy ends in
    handled after the loop).  Random lengths incl. 0 and odd ones, copylen =/</> csumlen.
    "src8": every source at +8 (payload after a 72-byte GM header); "mixed": some sources and
    some destinations byte-misaligned, interleaved in one batch.  (The names are round 1's, when
    these batches ran on 16-byte-piece streams.)"""
    rng = np.random.default_rng(n + len(layout))
    big = rng.random(n) < (0.5 if n == 40 else 0.05)
    cl = np.where(big, rng.integers(0, 300000, size=n), rng.integers(0, 5000, size=n))
    kind = rng.integers(0, 3, size=n)
    short = (cl * rng.random(n)).astype(np.int64)
    copylen = np.where(kind == 1, short, cl)
    csumlen = np.where(kind == 2, short, cl)
    sa = np.zeros(n, np.int64)
    da = np.zeros(n, np.int64)
    if layout == "src8":
        sa[:] = 8
    elif layout == "mixed":
        sa[::16] = rng.integers(1, 16, size=sa[::16].size)
        da[5::23] = rng.integers(1, 16, size=da[5::23].size)
    parts = np.zeros(n, np.uint64)
    got, want, dgot, dwant = _run(cuda, oracle, copylen, csumlen, sa, da, parts, 1)
    _assert_same(got, want, dgot, dwant, lambda i: (int(copylen[i]), int(csumlen[i]), int(sa[i]), int(da[i])))


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
@pytest.mark.parametrize("dst_align", [4, 8, 12])
def test_bcopy_batch_word_misaligned_dst(cuda, oracle, mode, dst_align):
    """Destinations 4, 8 or 12 bytes past a 16-byte boundary (the send side gathers payloads into
    GM ring slots right after the 72-byte header): in CRC mode whole rows go through the staged
    coalesced stores with the carried bytes, edge rows through word stores.  Multi-row fragments,
    ragged lengths, copylen =/</> csumlen, sources aligned or not; untouched bytes stay."""
    rng = np.random.default_rng(900 + dst_align + mode)
    n = 600
    cl = np.where(rng.random(n) < 0.3, rng.integers(0, 70000, size=n), 4096 * rng.integers(1, 9, size=n))
    kind = rng.integers(0, 3, size=n)
    short = (cl * rng.random(n)).astype(np.int64)
    copylen = np.where(kind == 1, short, cl)
    csumlen = np.where(kind == 2, short, cl)
    sa = np.where(rng.random(n) < 0.5, 0, rng.integers(0, 16, size=n))
    da = np.full(n, dst_align)
    parts = rng.integers(0, 2**32, size=n, dtype=np.uint64)
    got, want, dgot, dwant = _run(cuda, oracle, copylen, csumlen, sa, da, parts, mode)
    _assert_same(got, want, dgot, dwant, lambda i: (int(copylen[i]), int(csumlen[i]), int(sa[i]), int(da[i])))


def test_bcopy_batch_uniform_4k(cuda, oracle):
    """256K x 4 KiB gather into a staging array (the send-side shape): checksums vs the oracle,
    the copy compared on the device."""
    import torch

    dv = _dv()
    n, L = 262144, 4096
    src = torch.empty(n * L, dtype=torch.uint8, device=cuda)
    dv.fill_stream(src, seed=2)
    dst = torch.zeros(n * L, dtype=torch.uint8, device=cuda)
    # scatter: fragment i goes to slot perm[i]
    perm = np.random.default_rng(5).permutation(n).astype(np.uint64)
    offs = np.arange(n, dtype=np.uint64) * L
    descs = dv.make_copy_descs(src, offs, dst, perm * L, np.full(n, L), np.full(n, L))
    for mode in (0, 1):
        got = dv.as_u32(dv.frag_bcopy_batch(descs, mode=mode))
        assert np.array_equal(got, oracle.uniform_batch(2, 0, n, L, mode))
    assert torch.equal(dst.view(n, L)[torch.from_numpy(perm.astype(np.int64)).to(cuda)], src.view(n, L))


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
@pytest.mark.parametrize("msg_len,frag_len,stride,dst_off", [
    (4096 * 50000, 4096, 4096, 0),          # regular fast path, plain copy
    (4096 * 20000, 4096, 8192, 0),          # regular, staging slots with gaps
    (16384 * 3000, 16384, 16384 + 64, 16),  # regular, 4-row fragments
    (16384 * 3001, 16384, 16384 + 16, 0),   # regular, a last wave with an odd fragment count
    (4096 * 4097, 4096, 4096 + 32, 0),      # regular, 4 KiB, odd count in the last wave
    (65456 * 300 + 17, 65456, 65528, 0),    # GM payload into 72 + 65456-byte slots (general path)
    (1000003, 4096, 4100, 3),               # ragged everything
    (65456 * 300 + 1000, 65456, 65536, 72),  # GM slots: payload after the 72-byte header (dst % 16 = 8)
    (4096 * 5000 + 17, 4096, 4096 + 80, 72),  # 4 KiB payloads into 72-byte-header slots, ragged tail
    (4096 * 20001, 4096, 4096 + 80, 72),    # regular kernel into 72-byte-header slots (dst % 16 = 8)
    (16384 * 3001, 16384, 16384 + 76, 4),   # regular, 16 KiB, slot stride and base only 4-byte aligned
    (5, 4096, 4096, 1),                     # one short fragment
    # SUM: fragments of 16 KiB and more that are not whole rows go through row items
    # (MsgRowCopySource: one 4 KiB row per item, sums added per fragment)
    (16385 * 2000 + 3, 16385, 16385 + 7, 1),  # 5 rows, the last 1 byte; byte-misaligned destinations
    (40000 * 1500 + 12345, 40000, 40000, 0),  # a short last fragment with fewer rows
    (20001 * 777, 20001, 20480, 8),           # odd length, destinations at +8
    # SUM: 16-byte-multiple fragments of 4 KiB and more go one workgroup per 4 KiB row
    # (sum_copy_row_kernel) -- whole-row fragments and those of >= 64 rows as one-row groups joined
    # (round 5): partial last rows, short last fragments, dword-aligned slots
    (65456 * 300, 65456, 65536, 72),          # GM send: 65,456-byte payloads after the 72-byte header
    (65456 * 200 + 4000, 65456, 65536 + 4, 4),  # a last fragment of 4,000 bytes (one partial row)
    (4112 * 3000, 4112, 4112 + 12, 12),       # a second row of 16 bytes per fragment
    (49152 * 100 + 4096 * 5, 49152, 49152, 0),  # a last fragment of 5 of its 12 rows (groups)
    ((1 << 18) * 9 + 4096 * 70 + 16, 1 << 18, (1 << 18) + 4, 4),  # 64-row fragments as groups, the last one 6 rows + 16 B
    ((300000 // 16 * 16) * 40 + 48, 300000 // 16 * 16, 300032, 0),  # 74 rows, not whole rows: groups
    # CRC: 16-byte-multiple messages of fragments >= 4 KiB take the table-light copy
    # (crc_light_copy_kernel: one row per wave; rows of longer fragments joined by crc_light_join_kernel)
    ((1 << 20) * 40 + 4096 * 3 + 48, 1 << 20, (1 << 20) + 76, 4),  # 256-row fragments, a 3-row last one
    (4096 * 100000, 4096, 4096 + 80, 72),       # 4 KiB payloads into GM-style slots, 100,000 rows
    (65456 * 4000 + 400, 65456, 65536, 72),     # a GM message with a 400-byte last fragment
    # fragments under 2 KiB (SUM: one 128-thread workgroup each, ragged tails)
    (1976 * 5000 + 3, 1976, 2048 + 4, 4),     # shared-memory-sized fragments, ragged tail
    (100 * 3000, 100, 128, 1),                # tiny fragments, byte-misaligned destinations
    # SUM, 64 B .. 1 KiB fragments over >= 256 whole 4 KiB rows (round 6: sum_row4k_copy_kernel), the tail after them
    (64 * 20000 + 17, 64, 64, 0),             # contiguous destination, a 17-byte last fragment
    (256 * 5000 + 100, 256, 256 + 16, 3),     # slots, byte-misaligned destinations
    (1024 * 1100, 1024, 1024 + 72, 72),       # 1 KiB payloads after a 72-byte header
    (512 * 2100 + 511, 512, 600, 1),          # a stride that is not a multiple of 16
])
def test_msg_bcopy(cuda, oracle, mode, msg_len, frag_len, stride, dst_off):
    """lampi_msg_bcopy: fragment k -> dst + k*stride with its checksum fused; gap bytes untouched."""
    import torch

    dv = _dv()
    msg = torch.empty(msg_len, dtype=torch.uint8, device=cuda)
    dv.fill_stream(msg, seed=13)
    n = (msg_len + frag_len - 1) // frag_len
    dst_bytes = dst_off + (n - 1) * stride + frag_len + 64
    dst = torch.empty(dst_bytes, dtype=torch.uint8, device=cuda)
    dv.fill_stream(dst, seed=14)
    want_dst = dst.cpu().numpy().copy()
    host = msg.cpu().numpy()
    offs = np.arange(n, dtype=np.uint64) * frag_len
    lens = np.minimum(frag_len, msg_len - offs.astype(np.int64)).astype(np.uint32)
    for k in range(n):
        a, ln = int(offs[k]), int(lens[k])
        want_dst[dst_off + k * stride:dst_off + k * stride + ln] = host[a:a + ln]
    got = dv.as_u32(dv.msg_bcopy(msg, frag_len, dst[dst_off:], stride, partial=0x0BADF00D, mode=mode))
    want = oracle.desc_batch(host, offs, lens, np.full(n, 0x0BADF00D, np.uint32) if mode == 0 else None, mode)
    _assert_same(got, want, dst.cpu().numpy(), want_dst, lambda i: (i, int(lens[i])))


def test_sum_copy_grid_loop(cuda):
    """SUM copies beyond one grid (2^22 workgroups): the workgroups of sum_copy_wg_kernel (descriptor
    items) and sum_copy_row_kernel (message rows) take several items each.  Checked against the
    read-only SUM kernels (lampi_frag_csum_batch / lampi_msg_csum, parity-tested against the
    oracle elsewhere) and the copied bytes against the source."""
    import torch

    dv = _dv()
    n = (1 << 22) + 4099  # descriptor items: 64-byte fragments, every 3rd copied only in part
    L = 64
    src = torch.empty(n * L, dtype=torch.uint8, device=cuda)
    dv.fill_stream(src, seed=31)
    dst = torch.zeros(n * L + 64, dtype=torch.uint8, device=cuda)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    copylens = np.where(np.arange(n) % 3 == 0, 37, L).astype(np.int64)
    descs = dv.make_copy_descs(src, offs, dst, offs + np.uint64(4), copylens, np.full(n, L))
    got = dv.as_u32(dv.frag_bcopy_batch(descs, mode=dv.SUM32))
    want = dv.as_u32(dv.frag_csum_batch(dv.make_descs(src, offs, np.full(n, L)), mode=dv.SUM32))
    assert np.array_equal(got, want)
    d = dst[4:4 + n * L].view(n, L)
    s = src.view(n, L)
    full = torch.from_numpy(np.arange(n) % 3 != 0).to(cuda)
    assert torch.equal(d[full], s[full])
    assert torch.equal(d[~full][:, :37], s[~full][:, :37])
    assert not bool(d[~full][:, 37:].any())  # the residue is checksummed, not copied
    del src, dst, descs, d, s

    nf = 900001  # message rows: 5 rows per 16,400-byte fragment (not whole rows: row items), 4,500,005 rows
    F = 16400
    msg = torch.empty(nf * F, dtype=torch.uint8, device=cuda)
    dv.fill_stream(msg, seed=32)
    out = torch.empty(nf * F + 16, dtype=torch.uint8, device=cuda)
    got = dv.as_u32(dv.msg_bcopy(msg, F, out[16:], F, mode=dv.SUM32))
    want = dv.as_u32(dv.msg_csum(msg, F, mode=dv.SUM32))
    assert np.array_equal(got, want)
    assert torch.equal(out[16:16 + nf * F], msg)
