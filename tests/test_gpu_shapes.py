"""Batch shapes learned on the device ("Batch shapes learned on the device").

Without LAMPI_CSUM_ROWS_HINT the library samples a stream's descriptor batches on the device
(census_kernel, every 16th call) and runs later batches of 8-16-row fragments with the row-group
schedule the hint would select.  The schedule may change between two calls with the same inputs, so
every call is checked: read-only CRC and SUM batches, fused copies (checksums and every destination
byte) and the receive step, over GM-shaped batches, a mixed batch in between (the shape changes under
the learned hint) and GM-shaped batches again -- all against the oracle on a stream of their own.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 300  # >= the census's 256-descriptor minimum


def _dv():
    from lampi_amd import device as dv

    return dv


def _batches(rng, size):
    """Two shapes over one source buffer: GM-like (28,673..65,536 bytes: 8-16 rows, mostly 65,456) and
    mixed (0..70,000 bytes)."""
    gm = np.where(rng.random(N) < 0.7, 65456, rng.integers(28673, 65537, size=N)).astype(np.uint64)
    mixed = rng.integers(0, 70001, size=N).astype(np.uint64)
    offs = rng.integers(0, size - 70001, size=N).astype(np.uint64)
    parts = rng.integers(0, 2**32, size=N, dtype=np.uint64)
    return {"gm": gm, "mixed": mixed}, offs, parts


SEQUENCE = ["gm"] * 20 + ["mixed"] * 3 + ["gm"] * 18


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_learned_shape_read_only(cuda, oracle, mode):
    import torch

    dv = _dv()
    rng = np.random.default_rng(71 + mode)
    size = 48 << 20
    base = torch.empty(size, dtype=torch.uint8, device=cuda)
    dv.fill_stream(base, seed=72)
    host = base.cpu().numpy()
    lens, offs, parts = _batches(rng, size)
    prepared = {}
    for k, ln in lens.items():
        descs = dv.make_descs(base, offs, ln, parts if mode == 0 else None)
        want = oracle.desc_batch(host, offs, ln, parts.astype(np.uint32) if mode == 0 else None, mode)
        prepared[k] = (descs, want)
    stream = torch.cuda.Stream(device=cuda)
    with torch.cuda.stream(stream):
        for i, k in enumerate(SEQUENCE):
            descs, want = prepared[k]
            got = dv.as_u32(dv.frag_csum_batch(descs, mode=mode, stream=stream))
            assert np.array_equal(got, want), (i, k, int(np.count_nonzero(got != want)))


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_learned_shape_copies(cuda, oracle, mode):
    import torch

    dv = _dv()
    rng = np.random.default_rng(81 + mode)
    size = 48 << 20
    src = torch.empty(size, dtype=torch.uint8, device=cuda)
    dv.fill_stream(src, seed=82)
    host = src.cpu().numpy()
    lens, offs, parts = _batches(rng, size)
    dst = torch.empty(N * 70016, dtype=torch.uint8, device=cuda)
    doffs = (np.arange(N, dtype=np.uint64) * 70016 + rng.integers(0, 16, size=N).astype(np.uint64))
    prepared = {}
    for k, ln in lens.items():
        # copy all but a ragged tail of some fragments (the residue is checksummed, not copied)
        cl = np.where(rng.random(N) < 0.2, ln - np.minimum(ln, rng.integers(0, 40, size=N).astype(np.uint64)), ln)
        descs = dv.make_copy_descs(src, offs, dst, doffs, cl, ln, parts if mode == 0 else None)
        want = oracle.desc_batch(host, offs, ln.astype(np.uint32), parts.astype(np.uint32) if mode == 0 else None,
                                 mode)
        want_dst = np.zeros(dst.numel(), np.uint8)
        for i in range(N):
            a, b, c = int(offs[i]), int(doffs[i]), int(cl[i])
            want_dst[b:b + c] = host[a:a + c]
        prepared[k] = (descs, want, torch.from_numpy(want_dst).to(cuda))
    stream = torch.cuda.Stream(device=cuda)
    with torch.cuda.stream(stream):
        for i, k in enumerate(SEQUENCE):
            descs, want, want_dst = prepared[k]
            dst.zero_()
            got = dv.as_u32(dv.frag_bcopy_batch(descs, mode=mode, stream=stream))
            assert np.array_equal(got, want), (i, k, int(np.count_nonzero(got != want)))
            assert torch.equal(dst, want_dst), (i, k)


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_learned_shape_receive(cuda, oracle, mode):
    """CopyToApp over GM-shaped slots: every verdict, checksum and app byte, with a few fragments whose
    expected checksum is wrong (mask bits exact) and app buffers shorter than some fragments."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(91 + mode)
    size = 48 << 20
    frag = torch.empty(size, dtype=torch.uint8, device=cuda)
    dv.fill_stream(frag, seed=92)
    host = frag.cpu().numpy()
    lens, offs, _ = _batches(rng, size)
    app = torch.empty(N * 70016, dtype=torch.uint8, device=cuda)
    aoffs = np.arange(N, dtype=np.uint64) * 70016
    prepared = {}
    for k, ln in lens.items():
        app_len = np.where(rng.random(N) < 0.1, ln.astype(np.int64) - 100, ln.astype(np.int64) + 5)
        csum = oracle.desc_batch(host, offs, ln.astype(np.uint32), None if mode == 1 else
                                 np.full(N, 0xFFFFFFFF, np.uint32), mode)
        # AppBufferLen <= 0: DataOK, nothing copied, the checksum of nothing (oracle.copy_to_app)
        none = app_len <= 0
        csum = np.where(none, np.uint32(0xFFFFFFFF if mode == 0 else 0), csum).astype(np.uint32)
        bad = (rng.random(N) < 0.05) & ~none
        expected = np.where(bad, csum ^ 0x00A4A400, csum).astype(np.uint32)
        descs = dv.make_recv_descs(frag, offs, app, aoffs, ln, app_len)
        copy = np.minimum(ln.astype(np.int64), np.maximum(app_len, 0))
        want_app = np.zeros(app.numel(), np.uint8)
        for i in range(N):
            if not bad[i]:
                a, b, c = int(offs[i]), int(aoffs[i]), int(copy[i])
                want_app[b:b + c] = host[a:a + c]
        want_copied = np.where(bad, -1, copy)
        prepared[k] = (descs, torch.from_numpy(expected.view(np.int32)).to(cuda), csum, bad, want_copied,
                       torch.from_numpy(want_app).to(cuda))
    stream = torch.cuda.Stream(device=cuda)
    with torch.cuda.stream(stream):
        for i, k in enumerate(SEQUENCE):
            descs, expected, csum, bad, want_copied, want_app = prepared[k]
            app.zero_()
            copied, got, mask, nbad = dv.copy_to_app_batch(descs, expected, mode=mode, stream=stream)
            assert np.array_equal(dv.as_u32(got), csum), (i, k)
            assert np.array_equal(dv.mask_bits(mask, N), bad), (i, k)
            assert int(nbad.item()) == int(bad.sum()), (i, k)
            assert np.array_equal(copied.cpu().numpy(), want_copied), (i, k)
            # (a corrupt fragment's bytes may or may not have reached the app buffer: compare the good ones)
            good = torch.from_numpy(np.repeat(~bad, 70016)).to(cuda)
            assert torch.equal(app[good], want_app[good]), (i, k)


def _ib_lengths(rng, n, odd):
    """IB-sized fragments (16..2048 bytes, the half-frame edges among them); `odd`: a few fragments the
    pair kernel cannot take (0, 5, 15, 2049, 4096, 70,000 bytes) at indices the census does not sample,
    so the learned schedule still picks pairs and their workgroups run the per-fragment fallback."""
    edge = np.array([16, 17, 31, 32, 33, 1024, 1975, 1976, 2031, 2032, 2047, 2048], np.uint64)
    ln = np.where(rng.random(n) < 0.6, 1976, np.where(rng.random(n) < 0.5, rng.choice(edge, size=n),
                                                      rng.integers(16, 2049, size=n))).astype(np.uint64)
    if odd:
        sampled = set(int(x) for x in np.arange(64) * n // 64)
        free = [i for i in range(n) if i not in sampled]
        pick = rng.choice(free, size=12, replace=False)
        ln[pick] = rng.choice(np.array([0, 5, 15, 2049, 4096, 70000], np.uint64), size=12)
    return ln


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
@pytest.mark.parametrize("odd", [False, True], ids=["ib", "ib_odd"])
def test_learned_pairs_copies(cuda, oracle, odd, mode):
    """Copies of IB-sized fragments after the census: CRC two fragments to a wave (crc_light_pair_copy_kernel),
    SUM one fragment per wave four to a workgroup (sum_copy_waves_kernel); odd lengths, ragged copies
    (copylen < csumlen), misaligned sources and destinations, an odd count."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(101 + odd)
    n = 601
    ln = _ib_lengths(rng, n, odd)
    cl = np.where(rng.random(n) < 0.2, ln - np.minimum(ln, rng.integers(0, 24, size=n).astype(np.uint64)), ln)
    src = torch.empty(n * 70016 + 64, dtype=torch.uint8, device=cuda)
    dv.fill_stream(src, seed=102)
    host = src.cpu().numpy()
    offs = np.arange(n, dtype=np.uint64) * 70016 + rng.integers(0, 16, size=n).astype(np.uint64)
    dst = torch.empty(n * 70016 + 64, dtype=torch.uint8, device=cuda)
    doffs = np.arange(n, dtype=np.uint64) * 70016 + rng.integers(0, 16, size=n).astype(np.uint64)
    parts = rng.integers(0, 2**32, size=n, dtype=np.uint64)
    descs = dv.make_copy_descs(src, offs, dst, doffs, cl, ln, parts if mode == 0 else None)
    want = oracle.desc_batch(host, offs, ln.astype(np.uint32), parts.astype(np.uint32) if mode == 0 else None, mode)
    want_dst = np.zeros(dst.numel(), np.uint8)
    for i in range(n):
        a, b, c = int(offs[i]), int(doffs[i]), int(cl[i])
        want_dst[b:b + c] = host[a:a + c]
    want_dst = torch.from_numpy(want_dst).to(cuda)
    stream = torch.cuda.Stream(device=cuda)
    with torch.cuda.stream(stream):
        for i in range(20):
            dst.zero_()
            got = dv.as_u32(dv.frag_bcopy_batch(descs, mode=mode, stream=stream))
            assert np.array_equal(got, want), (i, [(int(j), int(ln[j])) for j in np.nonzero(got != want)[0][:8]])
            assert torch.equal(dst, want_dst), i


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
@pytest.mark.parametrize("odd", [False, True], ids=["ib", "ib_odd"])
def test_learned_pairs_receive(cuda, oracle, odd, mode):
    """CopyToApp of IB-sized fragments after the census picked pairs: checksums, verdicts (a few wrong
    expected values), AppBufferLen <= 0 / < / >= length, every delivered byte."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(111 + odd)
    n = 601
    ln = _ib_lengths(rng, n, odd)
    frag = torch.empty(n * 70016 + 64, dtype=torch.uint8, device=cuda)
    dv.fill_stream(frag, seed=112)
    host = frag.cpu().numpy()
    offs = np.arange(n, dtype=np.uint64) * 70016 + 8
    app = torch.empty(n * 70016, dtype=torch.uint8, device=cuda)
    aoffs = np.arange(n, dtype=np.uint64) * 70016 + rng.integers(0, 8, size=n).astype(np.uint64)
    app_len = np.where(rng.random(n) < 0.1, ln.astype(np.int64) - 30, ln.astype(np.int64) + 3)
    csum = oracle.desc_batch(host, offs, ln.astype(np.uint32), np.full(n, 0xFFFFFFFF, np.uint32) if mode == 0 else None,
                             mode)
    none = app_len <= 0
    csum = np.where(none, np.uint32(0xFFFFFFFF if mode == 0 else 0), csum).astype(np.uint32)
    bad = (rng.random(n) < 0.05) & ~none
    expected = np.where(bad, csum ^ 0x00A4A400, csum).astype(np.uint32)
    descs = dv.make_recv_descs(frag, offs, app, aoffs, ln, app_len)
    copy = np.minimum(ln.astype(np.int64), np.maximum(app_len, 0))
    want_app = np.zeros(app.numel(), np.uint8)
    for i in range(n):
        a, b, c = int(offs[i]), int(aoffs[i]), int(copy[i])
        want_app[b:b + c] = host[a:a + c]
    want_app = torch.from_numpy(want_app).to(cuda)
    exp_t = torch.from_numpy(expected.view(np.int32)).to(cuda)
    want_copied = np.where(bad, -1, copy)
    good = torch.from_numpy(np.repeat(~bad, 70016)).to(cuda)
    stream = torch.cuda.Stream(device=cuda)
    with torch.cuda.stream(stream):
        for i in range(20):
            app.zero_()
            copied, got, mask, nbad = dv.copy_to_app_batch(descs, exp_t, mode=mode, stream=stream)
            assert np.array_equal(dv.as_u32(got), csum), i
            assert np.array_equal(dv.mask_bits(mask, n), bad), i
            assert int(nbad.item()) == int(bad.sum()), i
            assert np.array_equal(copied.cpu().numpy(), want_copied), i
            assert torch.equal(app[good], want_app[good]), i


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_learned_pairs_shape_change(cuda, oracle, mode):
    """IB-sized copies until the census picks pairs, then batches of larger fragments on the same stream
    (the first of them still runs the pair schedule: every CRC wave leaves its fragments to the leftover
    kernel -- the list holds one entry per wave), then IB again."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(121 + mode)
    n = 601
    shapes = {"ib": _ib_lengths(rng, n, False),
              "big": rng.integers(2049, 70001, size=n).astype(np.uint64)}
    src = torch.empty(n * 70016 + 64, dtype=torch.uint8, device=cuda)
    dv.fill_stream(src, seed=122)
    host = src.cpu().numpy()
    offs = np.arange(n, dtype=np.uint64) * 70016 + rng.integers(0, 16, size=n).astype(np.uint64)
    dst = torch.empty(n * 70016 + 64, dtype=torch.uint8, device=cuda)
    doffs = np.arange(n, dtype=np.uint64) * 70016 + rng.integers(0, 16, size=n).astype(np.uint64)
    parts = rng.integers(0, 2**32, size=n, dtype=np.uint64)
    prepared = {}
    for k, ln in shapes.items():
        descs = dv.make_copy_descs(src, offs, dst, doffs, ln, ln, parts if mode == 0 else None)
        want = oracle.desc_batch(host, offs, ln.astype(np.uint32), parts.astype(np.uint32) if mode == 0 else None,
                                 mode)
        want_dst = np.zeros(dst.numel(), np.uint8)
        for i in range(n):
            a, b, c = int(offs[i]), int(doffs[i]), int(ln[i])
            want_dst[b:b + c] = host[a:a + c]
        prepared[k] = (descs, want, torch.from_numpy(want_dst).to(cuda))
    stream = torch.cuda.Stream(device=cuda)
    with torch.cuda.stream(stream):
        for i, k in enumerate(["ib"] * 20 + ["big"] * 4 + ["ib"] * 4):
            descs, want, want_dst = prepared[k]
            dst.zero_()
            got = dv.as_u32(dv.frag_bcopy_batch(descs, mode=mode, stream=stream))
            assert np.array_equal(got, want), (i, k, int(np.count_nonzero(got != want)))
            assert torch.equal(dst, want_dst), (i, k)


@pytest.mark.parametrize("L", [4096, 8192, 16384, 28672])
def test_learned_whole_row_descriptors(cuda, oracle, L):
    """Read-only CRC batches the census saw as equal whole-row fragments at 16-byte-aligned addresses run
    on the regular kernel (crc_regular_kernel<kDesc>, round 5): 4 KiB fragments in pairs, longer ones one
    per chain.  The same descriptor array then holds a batch where 1 in 20 fragments is not (lengths 0 / 1
    / L - 1 / L + 1 / 2L, odd addresses): under the stale shape those fragments (and their pair or even
    neighbour) are listed by the kernel and checksummed by the leftover launch.  Odd fragment counts end
    on the table-light kernel.  Every call vs the oracle."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(404 + L)
    n = 2 * 2048 * 2 + 1  # >= the path's minimum, odd
    size = max(64 << 20, n * (L + 64) * 2)
    base = torch.empty(size, dtype=torch.uint8, device=cuda)
    dv.fill_stream(base, seed=405)
    host = base.cpu().numpy()
    offs = (rng.integers(0, (size - 2 * L - 64) // 16, size=n) * 16).astype(np.uint64)
    parts = rng.integers(0, 2**32, size=n, dtype=np.uint64)
    full = np.full(n, L, np.uint64)
    odd_lens, odd_offs = full.copy(), offs.copy()
    pick = rng.choice(n, size=n // 20, replace=False)
    odd_lens[pick] = rng.choice(np.array([0, 1, L - 1, L + 1, 2 * L], np.uint64), size=pick.size)
    odd_offs[pick[::3]] += np.uint64(5)
    cases = {"full": (offs, full), "odd": (odd_offs, odd_lens)}
    prepared = {}
    for k, (o, ln) in cases.items():
        prepared[k] = (dv.make_descs(base, o, ln, parts),
                       oracle.desc_batch(host, o, ln.astype(np.uint32), parts.astype(np.uint32), 0))
    descs = prepared["full"][0].clone()  # one array whose contents change under its learned shape
    stream = torch.cuda.Stream(device=cuda)
    with torch.cuda.stream(stream):
        for i, k in enumerate(["full"] * 20 + ["odd"] * 4 + ["full"] * 3):
            descs.copy_(prepared[k][0])
            got = dv.as_u32(dv.frag_csum_batch(descs, mode=0, stream=stream))
            bad = np.nonzero(got != prepared[k][1])[0]
            assert bad.size == 0, (i, k, bad[:8].tolist())


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_learned_ib_pairs_read_only(cuda, oracle, mode):
    """Read-only batches of 1-2 KiB fragments (IB's 1,976-byte payloads) once the census has seen them (round
    5): CRC two to a wave on the table-light pair kernel (fragments ending off the 16-byte grid), SUM one per
    wave (sum_copy_waves_kernel).  The same descriptor array then holds fragments of other sizes (0 / 8 /
    2,049 / 4,096 / 9,000 bytes) under the stale shape: CRC lists their waves for the leftover launch, SUM's
    wave walks any length.  Every call vs the oracle."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(606)
    n = 3001
    size = 32 << 20
    base = torch.empty(size, dtype=torch.uint8, device=cuda)
    dv.fill_stream(base, seed=607)
    host = base.cpu().numpy()
    ib = np.where(rng.random(n) < 0.8, 1976, rng.integers(1025, 2049, size=n)).astype(np.uint64)
    offs = (rng.integers(0, (size - 16384) // 8, size=n) * 8).astype(np.uint64)
    parts = rng.integers(0, 2**32, size=n, dtype=np.uint64)
    odd = ib.copy()
    pick = rng.choice(n, size=n // 10, replace=False)
    odd[pick] = rng.choice(np.array([0, 8, 2049, 4096, 9000], np.uint64), size=pick.size)
    prepared = {k: (dv.make_descs(base, offs, ln, parts),
                    oracle.desc_batch(host, offs, ln.astype(np.uint32), parts.astype(np.uint32) if mode == 0 else None,
                                      mode))
                for k, ln in (("ib", ib), ("odd", odd))}
    descs = prepared["ib"][0].clone()
    stream = torch.cuda.Stream(device=cuda)
    with torch.cuda.stream(stream):
        for i, k in enumerate(["ib"] * 20 + ["odd"] * 4 + ["ib"] * 3):
            descs.copy_(prepared[k][0])
            got = dv.as_u32(dv.frag_csum_batch(descs, mode=mode, stream=stream))
            bad = np.nonzero(got != prepared[k][1])[0]
            assert bad.size == 0, (i, k, bad[:8].tolist())


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_learned_small_fragments_stale_shape(cuda, oracle, mode):
    """large batches the census saw as all-small (every sampled fragment <= 1 KiB / <= 2 KiB) run the
    piece streams with 256 fragments per workgroup (CRC, SUM) -- a schedule picked from a learned shape that can
    be stale.  70,000 descriptors of 64 B .. 1 KiB on one array for 20 calls, then the same array holding 0 B,
    17 B, 9,000 B and 1 MiB fragments at odd addresses among them; every call vs the oracle."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(707 + mode)
    n = 70_000
    size = 96 << 20
    base = torch.empty(size, dtype=torch.uint8, device=cuda)
    dv.fill_stream(base, seed=708)
    host = base.cpu().numpy()
    small = rng.integers(64, 1025, size=n).astype(np.uint64)
    offs = rng.integers(0, size - (1 << 20) - 1, size=n).astype(np.uint64)
    parts = rng.integers(0, 2**32, size=n, dtype=np.uint64)
    odd = small.copy()
    pick = rng.choice(n, size=n // 50, replace=False)
    odd[pick] = rng.choice(np.array([0, 17, 9000, 1 << 20], np.uint64), size=pick.size)
    odd_offs = offs.copy()
    odd_offs[pick] |= np.uint64(1)
    prepared = {k: (dv.make_descs(base, o, ln, parts),
                    oracle.desc_batch(host, o, ln.astype(np.uint32), parts.astype(np.uint32) if mode == 0 else None,
                                      mode))
                for k, (o, ln) in (("small", (offs, small)), ("odd", (odd_offs, odd)))}
    descs = prepared["small"][0].clone()
    stream = torch.cuda.Stream(device=cuda)
    with torch.cuda.stream(stream):
        for i, k in enumerate(["small"] * 20 + ["odd"] * 3 + ["small"] * 2):
            descs.copy_(prepared[k][0])
            got = dv.as_u32(dv.frag_csum_batch(descs, mode=mode, stream=stream))
            bad = np.nonzero(got != prepared[k][1])[0]
            assert bad.size == 0, (i, k, bad[:8].tolist())


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
@pytest.mark.parametrize("frag_len", [64, 100, 1000, 1024])
def test_small_fragment_messages_ragged(cuda, oracle, mode, frag_len):
    """Messages of >= 65,536 fragments of at most 1 KiB (the SUM piece streams at 256 fragments per workgroup,
    CRC's small-fragment schedules) with an odd start address and a ragged last fragment, vs the oracle."""
    import torch

    dv = _dv()
    n = 70_001
    msg_len = (n - 1) * frag_len + frag_len // 3 + 1
    buf = torch.empty(msg_len + 5, dtype=torch.uint8, device=cuda)
    dv.fill_stream(buf, seed=709)
    msg = buf[5:]
    got = dv.as_u32(dv.msg_csum(msg, frag_len, partial=0x1234567 if mode == 0 else 0xFFFFFFFF, mode=mode))
    host = buf.cpu().numpy()
    offs = 5 + np.arange(n, dtype=np.uint64) * frag_len
    lens = np.minimum(frag_len, msg_len + 5 - offs).astype(np.uint32)
    want = oracle.desc_batch(host, offs, lens, np.full(n, 0x1234567, np.uint32) if mode == 0 else None, mode)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
@pytest.mark.parametrize("L", [64, 256, 1024, 2048])
def test_learned_contiguous_descriptors_packed(cuda, oracle, L, mode):
    """Round 6: read-only descriptor batches the census saw as one contiguous run of equal L-byte fragments run as
    packed rows (crc_regular_kernel<kSub> from d[0].addr, each wave checking its items' descriptors; CRC up to 2 KiB,
    SUM up to 1 KiB, the leftovers on crc_light_pair_leftover_kernel / sum_pair_leftover_kernel).  The same
    array then holds, under the stale shape: a few descriptors moved elsewhere (odd addresses), with another length
    or another register; a batch that is not contiguous at all; a batch at another start; a shorter batch -- every
    call vs the oracle (items holding any of those go to the leftover launch; nothing outside the fragments is read)."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(800 + L)
    n = max(300 * 4096 // L, 600) + 37  # whole 8 KiB items plus a tail
    size = n * L + (8 << 20)
    base = torch.empty(size, dtype=torch.uint8, device=cuda)
    dv.fill_stream(base, seed=801)
    host = base.cpu().numpy()
    part = np.full(n, 0xFFFFFFFF, np.uint64)
    run = (np.arange(n, dtype=np.uint64) * np.uint64(L), np.full(n, L, np.uint64), part)
    moved = [a.copy() for a in run]
    pick = rng.choice(n, size=n // 200 + 3, replace=False)
    moved[0][pick[0::3]] = (rng.integers(0, size - 2 * L, size=pick[0::3].size) | 1).astype(np.uint64)
    moved[1][pick[1::3]] = rng.choice(np.array([0, 1, L - 1, L + 1, 3000], np.uint64), size=pick[1::3].size)
    moved[2][pick[2::3]] = rng.integers(0, 2**32, size=pick[2::3].size, dtype=np.uint64)
    scattered = (rng.integers(0, (size - L) // 16, size=n).astype(np.uint64) * np.uint64(16),
                 np.full(n, L, np.uint64), part)
    shifted = (run[0] + np.uint64(4096), run[1], part)
    cases = {"run": run, "moved": moved, "scattered": scattered, "shifted": shifted}
    prepared = {}
    for k, (o, ln, pt) in cases.items():
        prepared[k] = (dv.make_descs(base, o, ln, pt),
                       oracle.desc_batch(host, o, ln.astype(np.uint32), pt.astype(np.uint32) if mode == 0 else None,
                                         mode))
    descs = prepared["run"][0].clone()
    stream = torch.cuda.Stream(device=cuda)
    seq = ["run"] * 20 + ["moved"] * 3 + ["run"] * 2 + ["scattered"] * 2 + ["shifted"] * 2 + ["run"]
    with torch.cuda.stream(stream):
        for i, k in enumerate(seq):
            descs.copy_(prepared[k][0])
            got = dv.as_u32(dv.frag_csum_batch(descs, mode=mode, stream=stream))
            bad = np.nonzero(got != prepared[k][1])[0]
            assert bad.size == 0, (i, k, bad[:8].tolist())
        # a shorter batch on the same array (its first two thirds) under the learned shape
        m = n - n // 3
        got = dv.as_u32(dv.frag_csum_batch(descs, n=m, mode=mode, stream=stream))
        assert np.array_equal(got[:m], prepared["run"][1][:m])


def test_config_a_shape_descriptors_digest(cuda):
    """Config A's workload (1M x 1 KiB, stream seed 1) as one descriptor per fragment, after the census has seen
    it (packed rows): BASELINE.md's digest feb61101 / 41fadf13."""
    import torch

    from oracle.oracle import digest

    dv = _dv()
    n, L = 1048576, 1024
    buf = torch.empty(n * L, dtype=torch.uint8, device=cuda)
    dv.fill_stream(buf, seed=1)
    descs = dv.make_descs(buf, np.arange(n, dtype=np.uint64) * np.uint64(L), np.full(n, L, np.uint64))
    out = torch.empty(n, dtype=torch.int32, device=cuda)
    for _ in range(3):
        dv.frag_csum_batch(descs, out=out)
        assert digest(dv.as_u32(out)) == (0xFEB61101, 0x41FADF13)


def _ragged_layout(rng, lens, align=64):
    """Offsets of fragments laid one after another, each start rounded up to `align` (plus a random 0-2 blocks of gap)."""
    offs = np.empty(lens.size, np.uint64)
    o = 0
    for i, ln in enumerate(lens.tolist()):
        o = (o + align - 1) // align * align + align * int(rng.integers(0, 3))
        offs[i] = o
        o += ln
    return offs, o


@pytest.mark.parametrize("case", ["zipf", "bytes"])
def test_learned_ragged_descriptors(cuda, oracle, case):
    """Round 6: read-only CRC descriptor batches of mixed lengths up to 16 rows at 64-byte-aligned
    addresses, under whatever schedule the learned shape selects (the piece streams; the ragged whole-row kernel of
    commit dcda139 passed this test and was not adopted).  `zipf`: config C's lengths (64-byte
    multiples); `bytes`: any length 1 .. 65,536 (the ragged 1-7-row lengths 4,097 .. 28,671 among them) with random
    registers.  Then, on the same array under the learned shape: some descriptors moved off the 64-byte grid (odd and
    16-byte-aligned addresses), emptied or lengthened past 16 rows; the same lengths at odd addresses (1-byte
    alignment); a shorter batch -- every call vs the oracle."""
    import torch

    from lampi_amd.workload import zipf_lengths

    dv = _dv()
    rng = np.random.default_rng(9100 + len(case))
    if case == "zipf":
        lens = zipf_lengths(48 << 20).astype(np.uint64)
    else:
        n0 = 9000
        lens = np.concatenate([
            rng.integers(4097, 28672, size=n0 // 3),           # 2-7 rows, any length
            rng.integers(1, 4097, size=n0 // 3),                # one row
            rng.integers(28672, 65537, size=n0 // 6),           # 8-16 rows
            np.array([1, 2, 3, 4, 5, 63, 64, 65, 127, 128, 4095, 4096, 4097, 4159, 4160, 8191, 8192, 28671,
                      65535, 65536] * 20)]).astype(np.uint64)
        lens = lens[rng.permutation(lens.size)]
    n = lens.size
    offs, total = _ragged_layout(rng, lens)
    size = total + (1 << 20)
    base = torch.empty(size, dtype=torch.uint8, device=cuda)
    dv.fill_stream(base, seed=9101)
    host = base.cpu().numpy()
    part = (np.full(n, 0xFFFFFFFF, np.uint64) if case == "zipf"
            else rng.integers(0, 2**32, size=n, dtype=np.uint64))
    moved = [offs.copy(), lens.copy(), part]
    pick = rng.choice(n, size=n // 100 + 4, replace=False)
    moved[0][pick[0::4]] = (rng.integers(0, size - 70000, size=pick[0::4].size) | 1).astype(np.uint64)
    moved[0][pick[1::4]] = (rng.integers(0, (size - 70000) // 64, size=pick[1::4].size) * 64 + 16).astype(np.uint64)
    moved[1][pick[2::4]] = 0
    moved[0][pick[3::4]] = 0
    moved[1][pick[3::4]] = rng.integers(65537, 70001, size=pick[3::4].size).astype(np.uint64)
    odd = (np.minimum(offs + np.uint64(1), np.uint64(size) - lens), lens, part)
    cases = {"run": (offs, lens, part), "moved": tuple(moved), "odd": odd}
    prepared = {}
    for k, (o, ln, pt) in cases.items():
        prepared[k] = (dv.make_descs(base, o, ln, pt),
                       oracle.desc_batch(host, o, ln.astype(np.uint32), pt.astype(np.uint32), 0))
    descs = prepared["run"][0].clone()
    stream = torch.cuda.Stream(device=cuda)
    seq = ["run"] * 20 + ["moved"] * 3 + ["run"] * 2 + ["odd"] * 2 + ["run"]
    with torch.cuda.stream(stream):
        for i, k in enumerate(seq):
            descs.copy_(prepared[k][0])
            got = dv.as_u32(dv.frag_csum_batch(descs, mode=dv.CRC32, stream=stream))
            bad = np.nonzero(got != prepared[k][1])[0]
            assert bad.size == 0, (case, i, k, bad[:8].tolist(), lens[bad[:8]].tolist())
        m = n - n // 3
        got = dv.as_u32(dv.frag_csum_batch(descs, n=m, mode=dv.CRC32, stream=stream))
        assert np.array_equal(got[:m], prepared["run"][1][:m])


@pytest.mark.parametrize("L", [64, 256, 1024])
def test_learned_small_copy_descriptors_sum(cuda, oracle, L):
    """Round 6: SUM fused copies of descriptor batches of equal L-byte fragments (a message's fragments into slots) run
    one short-lived workgroup per 4 KiB of them once the census has seen the shape (sum_row4k_copy_desc_kernel); then,
    under that shape, descriptors with another copylen (0, 1, L - 1), a csumlen past L (residue checksummed, not
    copied) or a longer fragment (listed for sum_copy_list_kernel), and a shorter batch -- every sum and every
    destination byte (slot gaps untouched) vs the oracle."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(5100 + L)
    n = 300 * (4096 // L) + 37
    stride = L + 48
    src = torch.empty(n * L + 8192, dtype=torch.uint8, device=cuda)
    dv.fill_stream(src, seed=5101)
    hsrc = src.cpu().numpy()
    so = np.arange(n, dtype=np.uint64) * np.uint64(L)
    do = np.arange(n, dtype=np.uint64) * np.uint64(stride) + np.uint64(5)
    cl = np.full(n, L, np.int64)
    ck = np.full(n, L, np.int64)
    odd_cl, odd_ck = cl.copy(), ck.copy()
    pick = rng.choice(n, size=n // 50 + 3, replace=False)
    odd_cl[pick[0::3]] = rng.choice(np.array([0, 1, L - 1]), size=pick[0::3].size)
    odd_ck[pick[1::3]] = L + 7
    odd_cl[pick[2::3]] = L + 16
    odd_ck[pick[2::3]] = L + 16
    cases = {"run": (cl, ck), "odd": (odd_cl, odd_ck)}
    dst_bytes = int(do[-1]) + 2 * L + 64
    dst = torch.zeros(dst_bytes, dtype=torch.uint8, device=cuda)
    prepared = {k: dv.make_copy_descs(src, so, dst, do, c, s) for k, (c, s) in cases.items()}
    descs = prepared["run"].clone()  # one descriptor array: the census keys its shape on it
    stream = torch.cuda.Stream(device=cuda)
    seq = ["run"] * 20 + ["odd"] * 2 + ["run"]
    with torch.cuda.stream(stream):
        for i, k in enumerate(seq):
            c, s = cases[k]
            dst.zero_()
            descs.copy_(prepared[k])
            got = dv.as_u32(dv.frag_bcopy_batch(descs, mode=dv.SUM32, stream=stream))
            want = oracle.desc_batch(hsrc, so, np.maximum(c, s).astype(np.uint32), None, 1)
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, (L, i, k, bad[:8].tolist())
            stream.synchronize()
            hd = dst.cpu().numpy()
            want_dst = np.zeros(dst_bytes, np.uint8)
            for j in range(n):
                a, ln, b = int(so[j]), int(c[j]), int(do[j])
                want_dst[b:b + ln] = hsrc[a:a + ln]
            assert np.array_equal(hd, want_dst), (L, i, k)
