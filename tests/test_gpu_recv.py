"""GPU parity of the batched receive step RecvDesc_t::CopyToApp (lampi_copy_to_app_batch).

Ref src/path/common/BaseDesc.cc:288-342 (locked twin :380-434) with the GM hooks CopyFunction
(src/path/gm/recvFrag.h:165-182) and CheckData (:213-257): copy min(length_m, AppBufferLen)
bytes, checksum all length_m bytes, compare with header.dataChecksum unless nothing was copied,
AppBufferLen <= 0 = DataOK with nothing copied; return bytes copied or -1.

Expected values: oracle.oracle.copy_to_app, a composition of the reference-pinned bcopy_uicrc /
bcopy_uicsum restatement (the reference's own CopyToApp needs the whole path layer to build,
SURVEY.md 8(c), so the composition is pinned through its parts: tests/golden bcopy fixtures).
Fragments sit in GM-shaped NIC buffers: a 72-byte gmHeaderData whose dataChecksum (@64) is the
expected value, the payload right behind it (8-byte aligned), as gmFragBuffer lays them out
(src/path/gm/state.h:48-57, header.h:56-70).  Corruption follows the reference's injection,
dataChecksum |= 0xA4A4 (recvFrag.h:215-229).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HDR, DCSUM_OFF = 72, 64


def _dv():
    from lampi_amd import device as dv

    return dv


def _batch(rng, n, lengths=None):
    if lengths is None:
        pick = rng.integers(0, 6, size=n)
        lengths = np.where(pick == 0, rng.integers(0, 64, size=n),
                  np.where(pick == 1, rng.integers(64, 4200, size=n),
                  np.where(pick == 2, 4096,
                  np.where(pick == 3, 1976,
                  np.where(pick == 4, rng.integers(4096, 70000, size=n), 65456)))))
    lengths = np.asarray(lengths, dtype=np.int64)
    # AppBufferLen: <= 0, shorter than, equal to, longer than the fragment
    kind = rng.integers(0, 6, size=n)
    app_len = np.where(kind == 0, -rng.integers(0, 5000, size=n),
              np.where(kind == 1, 0,
              np.where(kind == 2, np.maximum(1, (lengths * rng.random(n)).astype(np.int64)),
              np.where(kind == 3, lengths, lengths + rng.integers(1, 1 << 40, size=n))))).astype(np.int64)
    return lengths, app_len


def _run_case(cuda, oracle, mode, lengths, app_len, rng, app_misalign=True, corrupt_frac=0.1, rows_hint=0):
    import torch

    from oracle.oracle import copy_to_app, copy_to_app_nochecksum

    dv = _dv()
    usecrc = mode == dv.CRC32
    n = lengths.size
    # NIC buffers: 72-byte header + payload, slot stride a multiple of 8 (gmFragBuffer)
    slot = HDR + ((lengths + 7) // 8) * 8 + 8
    soff = np.concatenate([[0], np.cumsum(slot[:-1])]).astype(np.int64)
    nic = torch.empty(int(slot.sum()) + 64, dtype=torch.uint8, device=cuda)
    dv.fill_stream(nic, seed=int(rng.integers(0, 1 << 30)))
    host = nic.cpu().numpy()
    poff = soff + HDR
    # expected = the true checksum of the payload, corrupted with |= 0xA4A4 for some fragments
    exp = np.zeros(n, np.uint32)
    bad_want = np.zeros(n, bool)
    ref = []
    for i in range(n):
        L = int(lengths[i])
        frag = host[poff[i]:poff[i] + L]
        true = oracle.uicrc(frag, L) if usecrc else oracle.uicsum(frag, L)[0]
        e = true
        if rng.random() < corrupt_frac:
            e = true | 0xA4A4
        exp[i] = e
        r = (copy_to_app_nochecksum(frag, L, int(app_len[i])) if mode == dv.NONE else
             copy_to_app(oracle, frag, L, int(app_len[i]), e, usecrc))
        ref.append(r)
        bad_want[i] = r[0] == -1
    hv = host.copy()
    for i in range(n):
        hv[soff[i] + DCSUM_OFF:soff[i] + DCSUM_OFF + 4] = np.frombuffer(np.uint32(exp[i]).tobytes(), np.uint8)
    nic.copy_(torch.from_numpy(hv).to(cuda))
    # application buffers: each fragment's delivery area behind a gap, sentinel-filled
    room = np.maximum(0, np.minimum(lengths, app_len))
    gap = rng.integers(0, 16, size=n) if app_misalign else np.zeros(n, np.int64)
    aslot = room + gap + 16
    aoff = (np.concatenate([[0], np.cumsum(aslot[:-1])]) + gap).astype(np.int64)
    app = torch.full((int(aslot.sum()) + 64,), 0x5C, dtype=torch.uint8, device=cuda)
    descs = dv.make_recv_descs(nic, poff, app, aoff, lengths, app_len)
    copied, csum, mask, nbad = _call(dv, descs, nic, soff, slot, n, mode, rows_hint)
    got_copied = copied.cpu().numpy()
    got_csum = csum.cpu().numpy().view(np.uint32)
    want_copied = np.array([r[0] for r in ref], np.int64)
    want_csum = np.array([r[1] for r in ref], np.uint32)
    assert np.array_equal(got_copied, want_copied), np.nonzero(got_copied != want_copied)[0][:10]
    assert np.array_equal(got_csum, want_csum), np.nonzero(got_csum != want_csum)[0][:10]
    assert np.array_equal(dv.mask_bits(mask, n), bad_want)
    assert int(nbad.item()) == int(bad_want.sum())
    # delivered bytes: exactly min(length, AppBufferLen) copied (also for corrupt fragments --
    # the reference copies before it checks), every other application byte untouched
    want_app = np.full(app.numel(), 0x5C, np.uint8)
    for i in range(n):
        d = ref[i][2]
        if d.size:
            want_app[aoff[i]:aoff[i] + d.size] = d
    assert np.array_equal(app.cpu().numpy(), want_app)
    return bad_want


def _call(dv, descs, nic, soff, slot, n, mode, rows_hint=0):
    """Expected checksums read straight out of the NIC buffers' headers: dataChecksum of record i
    at soff[i] + 64.  Uniform slots are one strided array (a GM receive ring); slots of varying
    size are first gathered into an array of 72-byte headers on the device."""
    import torch

    if np.all(slot == slot[0]):
        return dv.copy_to_app_batch(descs, nic, expected_stride=int(slot[0]), expected_offset=int(soff[0]) + DCSUM_OFF,
                                    n=n, mode=mode, rows_hint=rows_hint)
    idx = torch.from_numpy(soff[:, None] + np.arange(HDR)[None, :]).to(nic.device)
    hdrs = nic[idx.reshape(-1)].contiguous()
    return dv.copy_to_app_batch(descs, hdrs, expected_stride=HDR, expected_offset=DCSUM_OFF, n=n, mode=mode,
                                rows_hint=rows_hint)


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_copy_to_app_random(cuda, oracle, mode):
    rng = np.random.default_rng(100 + mode)
    lengths, app_len = _batch(rng, 3000)
    bad = _run_case(cuda, oracle, mode, lengths, app_len, rng)
    assert bad.any() and not bad.all()


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_copy_to_app_edges(cuda, oracle, mode):
    """Zero-length fragments, AppBufferLen <= 0 / == 1 / == length - 1 / == length / > length,
    lengths around the 64-byte piece and 4 KiB row edges, corrupt and clean."""
    rng = np.random.default_rng(7 + mode)
    L = [0, 1, 3, 4, 5, 63, 64, 65, 1975, 1976, 2047, 2048, 2049, 4095, 4096, 4097, 8192, 65455, 65456, 65536]
    lengths, app_len = [], []
    for ln in L:
        for a in sorted({-1, 0, 1, ln - 1, ln, ln + 1, 1 << 33}):
            lengths.append(ln)
            app_len.append(a)
    _run_case(cuda, oracle, mode, np.array(lengths), np.array(app_len), rng, corrupt_frac=0.3)


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
@pytest.mark.parametrize("rows_hint", [3, 16])
def test_copy_to_app_row_groups(cuda, oracle, rows_hint, mode):
    """The receive step with LAMPI_CSUM_ROWS_HINT (GM: 16 for 65,456-byte payloads): row groups joined
    before the verdict -- the edge cases (AppBufferLen <= 0 .. > length, corrupt and clean), then GM-sized
    payloads and longer ones (groups of several rows), every copy, checksum and verdict vs the oracle."""
    rng = np.random.default_rng(31 + rows_hint)
    L = [0, 1, 3, 4, 5, 63, 64, 65, 1975, 1976, 2047, 2048, 2049, 4095, 4096, 4097, 8192, 65455, 65456, 65536, 200003]
    lengths, app_len = [], []
    for ln in L:
        for a in sorted({-1, 0, 1, ln - 1, ln, ln + 1, 1 << 33}):
            lengths.append(ln)
            app_len.append(a)
    _run_case(cuda, oracle, mode, np.array(lengths), np.array(app_len), rng, corrupt_frac=0.3, rows_hint=rows_hint)
    n = 300
    lengths = np.where(rng.random(n) < 0.7, 65456, rng.integers(0, 140000, size=n))
    bad = _run_case(cuda, oracle, mode, lengths, np.full(n, 1 << 20), rng, corrupt_frac=0.1, rows_hint=rows_hint)
    assert bad.any() and not bad.all()


@pytest.mark.parametrize("rows_hint", [0, 16])
def test_copy_to_app_checksum_off(cuda, oracle, rows_hint):
    """LAMPI_CSUM_NONE (doChecksum == false, ref src/path/gm/recvFrag.h:178-181, :231-232): the delivered
    bytes are exactly min(length, AppBufferLen) of every fragment (also those whose header checksum is
    corrupt), the checksum output 0, every fragment DataOK -- the edge lengths, a random batch, GM payloads
    (with and without the rows hint) and IB-sized payloads (the learned wave-per-fragment schedule)."""
    dv = _dv()
    rng = np.random.default_rng(77 + rows_hint)
    L = [0, 1, 3, 4, 5, 63, 64, 65, 1975, 1976, 2048, 4095, 4096, 4097, 65456, 200003]
    lengths, app_len = [], []
    for ln in L:
        for a in sorted({-1, 0, 1, ln - 1, ln, ln + 1, 1 << 33}):
            lengths.append(ln)
            app_len.append(a)
    bad = _run_case(cuda, oracle, dv.NONE, np.array(lengths), np.array(app_len), rng, corrupt_frac=0.5,
                    rows_hint=rows_hint)
    assert not bad.any()
    lengths, app_len = _batch(rng, 2000)
    _run_case(cuda, oracle, dv.NONE, lengths, app_len, rng, corrupt_frac=0.3, rows_hint=rows_hint)
    n = 600
    for _ in range(3):  # the same shape again: the learned schedule takes over
        _run_case(cuda, oracle, dv.NONE, np.full(n, 65456), np.full(n, 1 << 20), rng, corrupt_frac=0.3,
                  rows_hint=rows_hint)
        _run_case(cuda, oracle, dv.NONE, np.full(n, 1976), np.full(n, 1 << 20), rng, corrupt_frac=0.3,
                  rows_hint=rows_hint)


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_copy_to_app_uniform_gm_slots(cuda, oracle, mode):
    """The common case: 4 KiB fragments in 72-byte-header slots, posted buffer large enough."""
    rng = np.random.default_rng(55 + mode)
    n = 2048
    lengths = np.full(n, 4096)
    app_len = np.full(n, 1 << 20)
    _run_case(cuda, oracle, mode, lengths, app_len, rng, app_misalign=False, corrupt_frac=0.01)


def test_copy_to_app_rejects_bad_args(cuda):
    import torch

    dv = _dv()
    from lampi_amd._lib import lib

    b = torch.zeros(64, dtype=torch.int64, device=cuda)
    p = b.data_ptr()
    assert lib().lampi_copy_to_app_batch(p, 1, p, 4, p, p, p, p, 7, None) != 0          # bad mode
    assert lib().lampi_copy_to_app_batch(p, 1, None, 4, p, p, p, p, 0, None) != 0       # CRC needs expected
    assert lib().lampi_copy_to_app_batch(p, 0, None, 4, None, None, None, p, 2, None) == 0  # NONE: none needed
    assert lib().lampi_copy_to_app_batch(p, 1, p + 2, 4, p, p, p, p, 0, None) != 0      # misaligned expected
    assert lib().lampi_copy_to_app_batch(p, 1, p, 6, p, p, p, p, 0, None) != 0          # misaligned stride
    assert lib().lampi_copy_to_app_batch(p, 0, None, 4, None, None, None, p, 0, None) == 0  # empty batch
    torch.cuda.synchronize()
    assert dv is not None


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_copy_to_app_alternating_shapes(cuda, oracle, mode):
    """One stream alternating GM receive batches (65,456-byte payloads) and IB ones (1,976 bytes), each from
    its own descriptor array, 48 calls: the learned shapes are kept per descriptor array (round 5), so each
    batch runs its own schedule (row groups / two per wave); every call's copies, checksums and verdicts
    against the oracle (results never depend on the schedule)."""
    import torch

    from oracle.oracle import copy_to_app

    dv = _dv()
    rng = np.random.default_rng(900 + mode)
    usecrc = mode == dv.CRC32

    def build(n, L):
        slot = HDR + ((L + 7) // 8) * 8 + 8
        nic = torch.empty(n * slot + 64, dtype=torch.uint8, device=cuda)
        dv.fill_stream(nic, seed=int(rng.integers(0, 1 << 30)))
        host = nic.cpu().numpy()
        soff = np.arange(n, dtype=np.int64) * slot
        exp = np.zeros(n, np.uint32)
        want_copied = np.zeros(n, np.int64)
        want_csum = np.zeros(n, np.uint32)
        for i in range(n):
            frag = host[soff[i] + HDR:soff[i] + HDR + L]
            true = oracle.uicrc(frag, L) if usecrc else oracle.uicsum(frag, L)[0]
            exp[i] = true | 0xA4A4 if rng.random() < 0.05 else true
            host[soff[i] + DCSUM_OFF:soff[i] + DCSUM_OFF + 4] = np.frombuffer(np.uint32(exp[i]).tobytes(), np.uint8)
            r = copy_to_app(oracle, frag, L, 1 << 30, int(exp[i]), usecrc)
            want_copied[i], want_csum[i] = r[0], r[1]
        nic.copy_(torch.from_numpy(host).to(cuda))
        app = torch.zeros(n * L + 64, dtype=torch.uint8, device=cuda)
        descs = dv.make_recv_descs(nic, soff + HDR, app, np.arange(n, dtype=np.int64) * L, np.full(n, L),
                                   np.full(n, 1 << 30, np.int64))
        return dict(n=n, L=L, slot=slot, nic=nic, app=app, descs=descs, copied=torch.from_numpy(want_copied).to(cuda),
                    csum=torch.from_numpy(want_csum.view(np.int32)).to(cuda),
                    payload=nic[:n * slot].view(n, slot)[:, HDR:HDR + L])

    gm, ib = build(600, 65456), build(3000, 1976)
    for call in range(48):
        b = gm if call % 2 == 0 else ib
        b["app"].zero_()
        copied, csum, mask, nbad = dv.copy_to_app_batch(b["descs"], b["nic"], expected_stride=b["slot"],
                                                        expected_offset=DCSUM_OFF, n=b["n"], mode=mode)
        assert torch.equal(copied, b["copied"]), (call, b["L"])
        assert torch.equal(csum, b["csum"]), (call, b["L"])
        assert int(nbad.item()) == int((b["copied"] == -1).sum().item())
        assert torch.equal(b["app"][:b["n"] * b["L"]].view(b["n"], b["L"]), b["payload"]), (call, b["L"])
