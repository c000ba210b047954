"""GPU parity of the send step written in place (strided outputs, checksumming off).

The reference's GM send of one fragment (gmSendFragDesc::init, ref src/path/gm/sendFrag.cc:143-226):

  contiguous:  headerp->dataChecksum = bcopy_uicrc / bcopy_uicsum(src, payload, len, len)   (:147-151)
  typemap:     csum threaded through one bcopy per piece, headerp->dataChecksum = csum     (:157-216)
  checksum off: MEMCOPY_FUNC only, dataChecksum left as it was                              (:153-155, :185-187)
  then (doChecksum only) headerp->checksum = headerChecksum(headerp, sizeof(gmHeader) - 4, GM_HDR_WORDS)
                                                                                            (:219-225)

Here a whole ring of 64 KiB GM buffers (72-byte gmHeaderData + up to 65,456 payload bytes, ref
src/path/gm/header.h:56-70) is packed by the batched entry points on one stream: a contiguous message
(lampi_msg_bcopy_strided), typemap fragments (lampi_chain_csum_batch_strided) and descriptor copies
(lampi_frag_bcopy_batch_strided), each stamping dataChecksum @64 in place, then the header checksums
@68 in place (lampi_header_csum_batch_strided).  Checked against the oracle (the pinned restatement of
MemFunctions.cc and of BasePath_t::headerChecksum): every dataChecksum, the receiver's header test
(CRC: uicrc(header || stored, 72) == 0; SUM: the 18 words sum to twice the stored word, ref
src/path/gm/path.cc:364-393), every payload byte, and every other byte of the ring unchanged.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BUF, HDR, PAYLOAD, WORDS = 65536, 72, 65456, 18
DCSUM, HCSUM = 64, 68


def _dv():
    from lampi_amd import device as dv

    return dv


def _ring(cuda, nbuf, seed):
    """A ring of nbuf GM buffers with random header fields, the checksum word zeroed (a fresh header)."""
    import torch

    dv = _dv()
    ring = torch.empty(nbuf * BUF, dtype=torch.uint8, device=cuda)
    dv.fill_stream(ring, seed=seed)
    v = ring.view(nbuf, BUF)
    v[:, HCSUM:HCSUM + 4] = 0
    return ring, v


def _oracle_sum_chain(oracle, pieces):
    tot, pi, pl = 0, 0, 0
    for p in pieces:
        s, pi, pl = oracle.uicsum(p, p.size, pi, pl)
        tot = (tot + s) & 0xFFFFFFFF
    return tot


def _oracle_crc_chain(oracle, pieces, init=0xFFFFFFFF):
    c = init
    for p in pieces:
        c = oracle.uicrc(p, p.size, c)
    return c


@pytest.mark.parametrize("mode", [0, 1, 2], ids=["crc", "sum", "none"])
def test_gm_ring_packed_in_place(cuda, oracle, mode):
    import torch

    dv = _dv()
    rng = np.random.default_rng(600 + mode)
    # slots [0, n_msg): one contiguous message of 37 fragments, the last one short
    n_msg = 37
    msg_len = (n_msg - 1) * PAYLOAD + 12_345
    # slots [n_msg, n_msg + n_tm): typemap fragments gathered from scattered pieces
    n_tm = 24
    # slots [n_msg + n_tm, nbuf): descriptor copies of ragged lengths from anywhere
    n_desc = 40
    nbuf = n_msg + n_tm + n_desc
    ring, v = _ring(cuda, nbuf, seed=71 + mode)
    before = v.cpu().numpy().copy()

    msg = torch.empty(msg_len + 3, dtype=torch.uint8, device=cuda)
    dv.fill_stream(msg, seed=72)
    msg = msg[3:]  # an odd start address
    dv.msg_bcopy_strided(msg, PAYLOAD, ring[HDR:], BUF, ring, BUF, out_offset=DCSUM, mode=mode)

    src = torch.empty(8 << 20, dtype=torch.uint8, device=cuda)
    dv.fill_stream(src, seed=73)
    tm_pieces, first, so, do, ln = [], [0], [], [], []
    for f in range(n_tm):
        pos = (n_msg + f) * BUF + HDR
        end = pos + int(rng.integers(0, PAYLOAD + 1))
        while pos < end:
            k = int(min(end - pos, rng.choice([1, 7, 64, 500, 4096, 20000])))
            so.append(int(rng.integers(0, src.numel() - k)))
            do.append(pos)
            ln.append(k)
            pos += k
        first.append(len(ln))
    pieces = dv.make_copy_descs(src, np.array(so, np.uint64), ring, np.array(do, np.uint64),
                                np.array(ln, np.uint32), np.array(ln, np.uint32),
                                np.full(len(ln), 0xFFFFFFFF, np.uint32))
    first_t = torch.tensor(np.array(first, np.uint32).view(np.int32), device=cuda)
    dv.chain_csum_batch_strided(pieces, first_t, ring, BUF, offset=n_msg * BUF + DCSUM, mode=mode)

    d_lens = rng.integers(0, PAYLOAD + 1, size=n_desc).astype(np.uint32)
    d_lens[:4] = [0, 1, 3, PAYLOAD]
    d_src = rng.integers(0, src.numel() - PAYLOAD, size=n_desc).astype(np.uint64)
    d_dst = ((n_msg + n_tm + np.arange(n_desc)) * BUF + HDR).astype(np.uint64)
    cd = dv.make_copy_descs(src, d_src, ring, d_dst, d_lens, d_lens, np.full(n_desc, 0xFFFFFFFF, np.uint32))
    dv.frag_bcopy_batch_strided(cd, ring, BUF, offset=(n_msg + n_tm) * BUF + DCSUM, mode=mode)

    dv.header_csum_batch_strided(ring, nbuf, BUF, HDR - 4, WORDS, ring, BUF, offset=HCSUM, mode=mode)
    after = v.cpu().numpy()
    m = msg.cpu().numpy()
    s = src.cpu().numpy()

    want = before.copy()
    payloads = []
    for k in range(n_msg):
        p = m[k * PAYLOAD:min((k + 1) * PAYLOAD, msg_len)]
        payloads.append([p])
    for f in range(n_tm):
        payloads.append([s[so[j]:so[j] + ln[j]] for j in range(first[f], first[f + 1])])
    for i in range(n_desc):
        payloads.append([s[int(d_src[i]):int(d_src[i]) + int(d_lens[i])]])
    for b, parts in enumerate(payloads):
        p = np.concatenate(parts) if parts else np.empty(0, np.uint8)
        want[b, HDR:HDR + p.size] = p
        if mode == 2:
            continue  # checksumming off: neither checksum word is written
        dc = _oracle_crc_chain(oracle, parts) if mode == 0 else _oracle_sum_chain(oracle, parts)
        want[b, DCSUM:DCSUM + 4] = np.array([dc], "<u4").view(np.uint8)
        hc = oracle.header_checksum(want[b, :HDR].copy(), HDR - 4, WORDS, mode == 0)
        want[b, HCSUM:HCSUM + 4] = np.array([hc], "<u4").view(np.uint8)
    for b in range(nbuf):
        assert np.array_equal(after[b], want[b]), f"buffer {b}"
    if mode != 2:
        # the receiver's header test passes on every buffer (device and oracle)
        mask, nbad = dv.header_check_batch(ring, nbuf, BUF, HDR, WORDS, HCSUM, mode=mode)
        assert int(nbad.item()) == 0
        for b in range(nbuf):
            h = after[b, :HDR].copy()
            if mode == 0:
                assert oracle.uicrc(h, HDR) == 0
            else:
                w = h.view("<u4").astype(np.uint64)
                assert int(w.sum()) & 0xFFFFFFFF == (2 * int(w[HCSUM // 4])) & 0xFFFFFFFF


@pytest.mark.parametrize("mode", [0, 1])
def test_strided_outputs_equal_plain_outputs(cuda, mode):
    """The strided forms write exactly the plain forms' words and no other byte (out_stride 4 too)."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(11 + mode)
    n = 3000
    src = torch.empty(16 << 20, dtype=torch.uint8, device=cuda)
    dv.fill_stream(src, seed=5)
    lens = rng.integers(0, 9000, size=n).astype(np.uint32)
    so = rng.integers(0, src.numel() - 9000, size=n).astype(np.uint64)
    dst = torch.zeros(n * 9001, dtype=torch.uint8, device=cuda)
    do = (np.arange(n) * 9001).astype(np.uint64)
    cd = dv.make_copy_descs(src, so, dst, do, lens, lens, rng.integers(0, 2**32, size=n, dtype=np.uint64))
    plain = dv.as_u32(dv.frag_bcopy_batch(cd, mode=mode))
    for stride, off in [(4, 0), (12, 4), (72, 64), (65536, 68)]:
        rec = torch.full(((n - 1) * stride + off + 8,), 0x5A, dtype=torch.uint8, device=cuda)
        dv.frag_bcopy_batch_strided(cd, rec, stride, offset=off, mode=mode)
        r = rec.cpu().numpy()
        idx = off + np.arange(n) * stride
        got = np.stack([r[idx + j] for j in range(4)], axis=1).copy().view("<u4").ravel()
        assert np.array_equal(got, plain)
        keep = np.ones(r.size, bool)
        for j in range(4):
            keep[idx + j] = False
        assert np.all(r[keep] == 0x5A)


@pytest.mark.parametrize("api", ["frag", "msg", "chain"])
def test_copies_with_checksumming_off(cuda, oracle, api):
    """LAMPI_CSUM_NONE on the send side: the bytes are copied exactly (copylen of each descriptor, nothing past
    it), no output is written, a NULL output is accepted."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(21)
    src = torch.empty(4 << 20, dtype=torch.uint8, device=cuda)
    dv.fill_stream(src, seed=9)
    s = src.cpu().numpy()
    dst = torch.full((10 << 20,), 0xA5, dtype=torch.uint8, device=cuda)
    want = np.full(dst.numel(), 0xA5, np.uint8)
    if api == "frag":
        n = 5000
        cl = rng.integers(0, 700, size=n).astype(np.uint32)
        cl[::97] = rng.integers(4096, 70000, size=cl[::97].size)
        xl = cl + rng.integers(0, 64, size=n).astype(np.uint32)  # csumlen > copylen: not copied, not needed
        so = rng.integers(0, src.numel() - 70100, size=n).astype(np.uint64)
        do = np.concatenate([[0], np.cumsum(cl.astype(np.uint64) + 3)[:-1]]).astype(np.uint64)
        cd = dv.make_copy_descs(src, so, dst, do, cl, xl)
        assert dv.frag_bcopy_batch(cd, mode=dv.NONE) is None
        for a, b, c in zip(so, do, cl):
            want[int(b):int(b) + int(c)] = s[int(a):int(a) + int(c)]
    elif api == "msg":
        L, stride, mlen = 1976, 2048, 1976 * 700 + 55
        msg = src[1:1 + mlen]
        assert dv.msg_bcopy(msg, L, dst, stride, mode=dv.NONE) is None
        for k in range((mlen + L - 1) // L):
            c = min(L, mlen - k * L)
            want[k * stride:k * stride + c] = s[1 + k * L:1 + k * L + c]
    else:
        nfr, first, so, do, ln = 300, [0], [], [], []
        pos = 0
        for f in range(nfr):
            for _ in range(int(rng.integers(0, 9))):
                k = int(rng.integers(1, 3000))
                so.append(int(rng.integers(0, src.numel() - k)))
                do.append(pos)
                ln.append(k)
                pos += k
            pos += 5
            first.append(len(ln))
        pieces = dv.make_copy_descs(src, np.array(so, np.uint64), dst, np.array(do, np.uint64),
                                    np.array(ln, np.uint32), np.array(ln, np.uint32))
        assert dv.chain_csum_batch(pieces, first, mode=dv.NONE) is None
        for a, b, c in zip(so, do, ln):
            want[b:b + c] = s[a:a + c]
    assert np.array_equal(dst.cpu().numpy(), want)


def test_send_entry_points_reject_bad_outputs(cuda):
    import torch

    from lampi_amd import lib

    buf = torch.zeros(1 << 16, dtype=torch.uint8, device=cuda)
    p = buf.data_ptr()
    L = lib()
    # a checksum output is required unless checksumming is off; strides are 4-byte multiples >= 4
    assert L.lampi_frag_bcopy_batch_strided(p, 1, None, 72, 0, None) != 0
    assert L.lampi_frag_bcopy_batch_strided(p, 1, p + 2, 72, 0, None) != 0
    assert L.lampi_frag_bcopy_batch_strided(p, 1, p, 6, 0, None) != 0
    assert L.lampi_frag_bcopy_batch_strided(p, 1, p, 0, 1, None) != 0
    assert L.lampi_frag_bcopy_batch_strided(p, 1, p, 8, 3, None) != 0  # unknown mode
    assert L.lampi_msg_bcopy_strided(p, 100, 10, p + 4096, 16, 0, None, 72, 1, None) != 0
    assert L.lampi_msg_bcopy_strided(p, 100, 10, p + 4096, 8, 0, p, 72, 1, None) != 0  # slot stride < frag_len
    assert L.lampi_chain_csum_batch_strided(p, 0, p, 1, None, 4, 0, None) != 0
    assert L.lampi_header_csum_batch_strided(p, 4, 72, 68, 18, p + 1, 72, 0, None) != 0
    # checksumming off: no output needed, the header stamp is a no-op
    assert L.lampi_header_csum_batch_strided(p, 4, 72, 68, 18, None, 0, 2, None) == 0
    assert L.lampi_msg_bcopy_strided(p, 0, 10, p + 4096, 16, 0, None, 0, 2, None) == 0
    # the checksum-only entry points still refuse NONE
    assert L.lampi_msg_csum(p, 100, 10, 0, p + 4096, 2, None) != 0
    assert L.lampi_frag_csum_batch(p, 1, p + 4096, 2, None) != 0
    torch.cuda.synchronize()


def test_host_msg_bcopy_checksumming_off(cuda):
    """lampi_host_msg_bcopy with LAMPI_CSUM_NONE: the fragments land in the ring slots, h_out is not needed."""
    import ctypes

    from lampi_amd import lib

    rng = np.random.default_rng(3)
    L, stride, mlen = 65456, 65536, 65456 * 40 + 999
    msg = rng.integers(0, 256, size=mlen, dtype=np.uint8)
    ring = np.full(stride * 41, 0x3C, np.uint8)
    rc = lib().lampi_host_msg_bcopy(msg.ctypes.data, mlen, L, 2, 37, ring.ctypes.data_as(ctypes.c_void_p), stride,
                                    0xFFFFFFFF, None, 2)
    assert rc == 0
    want = np.full_like(ring, 0x3C)
    for i in range(37):
        k = 2 + i
        c = min(L, mlen - k * L)
        want[i * stride:i * stride + c] = msg[k * L:k * L + c]
    assert np.array_equal(ring, want)
