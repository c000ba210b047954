"""GPU parity of the header and receive-side verification batches.

  lampi_header_csum_batch   BasePath_t::headerChecksum (ref src/path/common/path.h:280-314)
  lampi_header_check_batch  receiver header check      (ref src/path/gm/path.cc:364-393)
  lampi_check_data_batch    CheckData                   (ref src/path/gm/recvFrag.h:213-257)

Header checksums are compared with the oracle's restatement of headerChecksum (whose CRC is
the reference-pinned uicrc).  The verification masks are compared bit-exact with the set of
records the test corrupted, on GM-shaped records: a 72-byte gmHeaderData (dataLength @20,
dataChecksum @64, checksum @68; ref src/path/gm/header.h:56-70) followed by its payload.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HDR, WORDS, DATALEN_OFF, DCSUM_OFF, HCSUM_OFF = 72, 18, 20, 64, 68


def _dv():
    from lampi_amd import device as dv

    return dv


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
@pytest.mark.parametrize("crclen,words,stride", [(68, 18, 72), (72, 18, 200), (124, 32, 128), (128, 32, 128),
                                                 (9, 2, 16), (71, 17, 1096)])
def test_header_checksums(cuda, oracle, mode, crclen, words, stride):
    import torch

    dv = _dv()
    n = 3000
    buf = torch.empty(n * stride + 64, dtype=torch.uint8, device=cuda)
    dv.fill_stream(buf, seed=71)
    got = dv.as_u32(dv.header_csum_batch(buf, n, stride, crclen, words, mode=mode))
    host = buf.cpu().numpy()
    want = np.array([oracle.header_checksum(host[i * stride:i * stride + max(crclen, 4 * words)], crclen, words,
                                            mode == 0) for i in range(n)], np.uint32)
    assert np.array_equal(got, want)


def _gm_records(cuda, n, payload, seed):
    """n GM-shaped records (72-byte header + payload); header words random, checksum field 0."""
    import torch

    dv = _dv()
    stride = HDR + payload
    rec = torch.empty(n * stride, dtype=torch.uint8, device=cuda)
    dv.fill_stream(rec, seed=seed)
    v = rec.view(n, stride)
    v[:, HCSUM_OFF:HCSUM_OFF + 4] = 0
    return rec, v, stride


def _put_u32(v, col, vals):
    import torch

    b = torch.from_numpy(np.ascontiguousarray(vals.astype("<u4")).view(np.uint8).reshape(-1, 4)).to(v.device)
    v[:, col:col + 4] = b


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_header_residue_and_corruption(cuda, mode):
    """Sender stamps headerChecksum over 68 bytes (sendFrag.cc:218-225); the receiver's check over
    the whole 72-byte header passes for every record and flags exactly the corrupted ones."""
    import torch

    dv = _dv()
    n = 20000
    rec, v, stride = _gm_records(cuda, n, 256, seed=72)
    csum = dv.as_u32(dv.header_csum_batch(rec, n, stride, HDR - 4, WORDS, mode=mode))
    _put_u32(v, HCSUM_OFF, csum)
    mask, nbad = dv.header_check_batch(rec, n, stride, HDR, WORDS, HCSUM_OFF, mode=mode)
    assert int(nbad.item()) == 0 and not dv.mask_bits(mask, n).any()

    rng = np.random.default_rng(5)
    bad = np.sort(rng.choice(n, size=777, replace=False))
    host = v.cpu().numpy()
    for k, i in enumerate(bad):
        if k % 5 == 0:  # the reference's artificial corruption: checksum |= 0xA4A4 (path.cc:352-357)
            w = int.from_bytes(host[i, HCSUM_OFF:HCSUM_OFF + 4].tobytes(), "little")
            w2 = w | 0xA4A4 if (w | 0xA4A4) != w else w ^ 0xA4A4
            host[i, HCSUM_OFF:HCSUM_OFF + 4] = np.frombuffer(w2.to_bytes(4, "little"), np.uint8)
        else:
            host[i, int(rng.integers(0, HDR))] ^= np.uint8(rng.integers(1, 256))
    v.copy_(torch.from_numpy(host).to(cuda))
    mask, nbad = dv.header_check_batch(rec, n, stride, HDR, WORDS, HCSUM_OFF, mode=mode)
    got = np.nonzero(dv.mask_bits(mask, n))[0]
    assert np.array_equal(got, bad)
    assert int(nbad.item()) == bad.size


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_receive_pipeline_check_data(cuda, mode):
    """Send side stamps dataLength/dataChecksum; receive side checksums the payloads (descriptor
    batch) and CheckData reads the expected values straight from the headers."""
    import torch

    dv = _dv()
    n, payload = 12000, 1976  # the IB payload size
    rec, v, stride = _gm_records(cuda, n, payload, seed=73)
    rng = np.random.default_rng(6)
    lens = rng.integers(0, payload + 1, size=n).astype(np.uint32)
    lens[::50] = 0
    offs = np.arange(n, dtype=np.uint64) * stride + HDR
    descs = dv.make_descs(rec, offs, lens)
    calc = dv.frag_csum_batch(descs, mode=mode)
    _put_u32(v, DATALEN_OFF, lens)
    _put_u32(v, DCSUM_OFF, dv.as_u32(calc))
    mask, nbad = dv.check_data_batch(calc, rec, stride, rec, stride, n=n, expected_offset=DCSUM_OFF,
                                     lengths_offset=DATALEN_OFF)
    assert int(nbad.item()) == 0

    # corrupt payload bytes of some nonempty fragments, then re-checksum as the receiver would
    host = v.cpu().numpy()
    cand = np.nonzero(lens > 0)[0]
    bad = np.sort(rng.choice(cand, size=321, replace=False))
    for i in bad:
        host[i, HDR + int(rng.integers(0, lens[i]))] ^= np.uint8(rng.integers(1, 256))
    # zero-length fragments with a garbage expected checksum still pass (recvFrag.h:235)
    zero = np.nonzero(lens == 0)[0]
    host[zero, DCSUM_OFF] ^= 0x5A
    v.copy_(torch.from_numpy(host).to(cuda))
    calc2 = dv.frag_csum_batch(descs, mode=mode)
    mask, nbad = dv.check_data_batch(calc2, rec, stride, rec, stride, n=n, expected_offset=DCSUM_OFF,
                                     lengths_offset=DATALEN_OFF)
    assert np.array_equal(np.nonzero(dv.mask_bits(mask, n))[0], bad)
    assert int(nbad.item()) == bad.size
    # without lengths every mismatch counts, including the zero-length ones
    mask, nbad = dv.check_data_batch(calc2, rec, stride, None, 4, n=n, expected_offset=DCSUM_OFF)
    assert np.array_equal(np.nonzero(dv.mask_bits(mask, n))[0], np.union1d(bad, zero))


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_checksums_stamped_into_headers(cuda, mode):
    """lampi_frag_csum_batch_strided writes checksum i into record i's dataChecksum field
    (gm/sendFrag.cc:147-155 stores it there) and leaves every other byte alone."""
    dv = _dv()
    n, payload = 9000, 1976
    rec, v, stride = _gm_records(cuda, n, payload, seed=74)
    rng = np.random.default_rng(9)
    lens = rng.integers(0, payload + 1, size=n).astype(np.uint32)
    descs = dv.make_descs(rec, np.arange(n, dtype=np.uint64) * stride + HDR, lens)
    want = dv.as_u32(dv.frag_csum_batch(descs, mode=mode))
    before = v.cpu().numpy().copy()
    dv.frag_csum_batch_strided(descs, rec, stride, offset=DCSUM_OFF, mode=mode)
    after = v.cpu().numpy()
    assert np.array_equal(after[:, DCSUM_OFF:DCSUM_OFF + 4].copy().view("<u4").ravel(), want)
    before[:, DCSUM_OFF:DCSUM_OFF + 4] = after[:, DCSUM_OFF:DCSUM_OFF + 4]
    assert np.array_equal(before, after)


def test_verify_rejects_misaligned(cuda):
    import torch

    import lampi_amd

    buf = torch.zeros(4096, dtype=torch.uint8, device=cuda)
    rc = lampi_amd.lib().lampi_header_csum_batch(buf.data_ptr() + 1, 4, 72, 68, 18, buf.data_ptr(), 0, None)
    assert rc != 0
    rc = lampi_amd.lib().lampi_header_check_batch(buf.data_ptr(), 4, 70, 72, 18, 68, buf.data_ptr(),
                                                  buf.data_ptr() + 64, 0, None)
    assert rc != 0
    rc = lampi_amd.lib().lampi_frag_csum_batch_strided(buf.data_ptr(), 4, buf.data_ptr() + 2, 72, 0, None)
    assert rc != 0
    rc = lampi_amd.lib().lampi_frag_csum_batch_strided(buf.data_ptr(), 4, buf.data_ptr(), 70, 0, None)
    assert rc != 0


# ---- the IB variant: uicrc/uicsum of the header stored unswapped and compared by the receiver ----
# ibDataHdr_t is 72 bytes with the header checksum last (ref src/path/ib/header.h:48-62); the sender
# stores uicrc(p, 68) / uicsum(p, 68) (src/path/ib/sendFrag.cc:306-314), an ACK uicrc(p, len - 4)
# (:327-335); the receiver recomputes over the same bytes and compares (src/path/ib/path.cc:652-680).
IB_BUF = 2048  # ibData2KMsg_t: header + 1,976 payload bytes (ib/header.h:75-80)


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
@pytest.mark.parametrize("crclen,stride", [(68, IB_BUF), (60, 64), (57, 64), (67, 1096)])
def test_ib_header_stamp_and_compare(cuda, oracle, mode, crclen, stride):
    """Sender (lampi_frag_csum_batch_strided over one descriptor per header, stored at crclen rounded up to
    a word) matches the oracle's uicrc/uicsum; the receiver check (lampi_header_compare_batch) passes every
    record and flags exactly the corrupted ones, including the reference's |= 0xA4A4 corruption."""
    import torch

    dv = _dv()
    n = 6000
    off = (crclen + 3) // 4 * 4  # where the sender keeps the checksum word
    rec = torch.empty(n * stride, dtype=torch.uint8, device=cuda)
    dv.fill_stream(rec, seed=90 + crclen)
    v = rec.view(n, stride)
    descs = dv.make_descs(rec, np.arange(n, dtype=np.uint64) * stride, np.full(n, crclen))
    dv.frag_csum_batch_strided(descs, rec, stride, offset=off, mode=mode)
    host = v.cpu().numpy()
    stored = host[:, off:off + 4].copy().view("<u4").ravel()
    if mode == 0:
        want = np.array([oracle.uicrc(host[i, :crclen], crclen) for i in range(n)], np.uint32)
    else:
        want = np.array([oracle.uicsum(host[i, :crclen], crclen)[0] for i in range(n)], np.uint32)
    assert np.array_equal(stored, want)
    mask, nbad = dv.header_compare_batch(rec, n, stride, crclen, off, mode=mode)
    assert int(nbad.item()) == 0 and not dv.mask_bits(mask, n).any()

    rng = np.random.default_rng(crclen)
    bad = np.sort(rng.choice(n, size=555, replace=False))
    for k, i in enumerate(bad):
        if k % 5 == 0:  # ENABLE_RELIABILITY's artificial corruption of the stored checksum
            w = int(stored[i])
            w2 = w | 0xA4A4 if (w | 0xA4A4) != w else w ^ 0xA4A4
            host[i, off:off + 4] = np.frombuffer(w2.to_bytes(4, "little"), np.uint8)
        else:  # a flipped byte in the checked header bytes
            host[i, int(rng.integers(0, crclen))] ^= np.uint8(rng.integers(1, 256))
    v.copy_(torch.from_numpy(host).to(cuda))
    mask, nbad = dv.header_compare_batch(rec, n, stride, crclen, off, mode=mode)
    assert np.array_equal(np.nonzero(dv.mask_bits(mask, n))[0], bad)
    assert int(nbad.item()) == bad.size
    # the bytes past crclen (e.g. the payload of an ibData2KMsg) are not part of the check
    if stride > off + 8:
        host[:, off + 4:] ^= np.uint8(0x5A)
        v.copy_(torch.from_numpy(host).to(cuda))
        mask, nbad = dv.header_compare_batch(rec, n, stride, crclen, off, mode=mode)
        assert np.array_equal(np.nonzero(dv.mask_bits(mask, n))[0], bad)


def test_ib_header_compare_rejects_bad_arguments(cuda):
    import torch

    import lampi_amd

    buf = torch.zeros(4096, dtype=torch.uint8, device=cuda)
    c = lampi_amd.lib()
    assert c.lampi_header_compare_batch(buf.data_ptr() + 1, 4, 72, 68, 68, buf.data_ptr(), buf.data_ptr(), 0, None) != 0
    assert c.lampi_header_compare_batch(buf.data_ptr(), 4, 70, 68, 68, buf.data_ptr(), buf.data_ptr(), 0, None) != 0
    assert c.lampi_header_compare_batch(buf.data_ptr(), 4, 72, 68, 66, buf.data_ptr(), buf.data_ptr(), 0, None) != 0
    assert c.lampi_header_compare_batch(buf.data_ptr(), 4, 72, 68, 68, buf.data_ptr(), buf.data_ptr(), 3, None) != 0
