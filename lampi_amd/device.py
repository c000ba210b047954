"""Device-resident batched checksums over torch CUDA tensors (HIP on ROCm).

PyTorch is only plumbing here: it owns HBM buffers and streams.  Every checksum is
computed by the gfx950 kernels behind the C ABI (lampi_frag_csum_batch, lampi_frag_bcopy_batch,
lampi_msg_csum).
"""
from __future__ import annotations

import numpy as np
import torch

from ._lib import BY_BYTES, CRC32, CRC_INITIAL_REGISTER, NONE, SUM32, check, lib, rows_hint_bits

__all__ = ["CRC32", "SUM32", "NONE", "chain_copy_to_app_batch", "frag_bcopy_batch_strided", "msg_bcopy_strided",
           "chain_csum_batch_strided", "header_csum_batch_strided", "frag_csum_batch", "diag_frag_csum_batch_per_wave", "frag_csum64_batch", "frag_bcopy_batch", "msg_bcopy", "msg_csum", "fill_stream", "fill_stream_frags",
           "make_descs", "make_copy_descs", "as_u32", "chain_csum_batch", "header_csum_batch", "header_check_batch", "check_data_batch",
           "mask_bits", "make_recv_descs", "copy_to_app_batch"]


def _stream_handle(stream: torch.cuda.Stream | None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def _require_cuda(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise ValueError(f"{what} must be a device (cuda) tensor")
    if not t.is_contiguous():
        raise ValueError(f"{what} must be contiguous")


def as_u32(t: torch.Tensor) -> np.ndarray:
    """Checksum tensor (int32 storage) -> numpy uint32 on the host."""
    return t.detach().cpu().numpy().view(np.uint32)


def make_descs(base: torch.Tensor, offsets, lengths, partials=None) -> torch.Tensor:
    """Build a device array of ``lampi_frag_desc`` (n x 16 bytes, int64 [n, 2] storage)."""
    _require_cuda(base, "base")
    off = np.asarray(offsets, dtype=np.uint64)
    ln = np.asarray(lengths, dtype=np.uint64)
    n = off.size
    if ln.size != n:
        raise ValueError("offsets and lengths differ in size")
    if n and int((off + ln).max()) > base.numel() * base.element_size():
        raise ValueError("a fragment extends past the end of the base tensor")
    if n and int(ln.max()) > 0xFFFFFFFF:
        raise ValueError("fragment length exceeds 32 bits")
    pt = (np.full(n, CRC_INITIAL_REGISTER, dtype=np.uint64) if partials is None
          else np.asarray(partials, dtype=np.uint64) & 0xFFFFFFFF)
    host = np.empty((n, 2), dtype=np.uint64)
    host[:, 0] = np.uint64(base.data_ptr()) + off
    host[:, 1] = ln | (pt << np.uint64(32))
    return torch.from_numpy(host.view(np.int64)).to(base.device)


def make_copy_descs(src: torch.Tensor, src_offsets, dst: torch.Tensor, dst_offsets, copylens, csumlens,
                    partials=None) -> torch.Tensor:
    """Build a device array of ``lampi_copy_desc`` (n x 32 bytes, int64 [n, 4] storage)."""
    _require_cuda(src, "src")
    _require_cuda(dst, "dst")
    so = np.asarray(src_offsets, dtype=np.uint64)
    do = np.asarray(dst_offsets, dtype=np.uint64)
    cl = np.asarray(copylens, dtype=np.uint64)
    sl = np.asarray(csumlens, dtype=np.uint64)
    n = so.size
    if not (do.size == cl.size == sl.size == n):
        raise ValueError("descriptor fields differ in size")
    if n:
        if int(np.maximum(cl, sl).max()) > 0xFFFFFFFF:
            raise ValueError("length exceeds 32 bits")
        if int((so + np.maximum(cl, sl)).max()) > src.numel() * src.element_size():
            raise ValueError("a source fragment extends past the end of src")
        if int((do + cl).max()) > dst.numel() * dst.element_size():
            raise ValueError("a copy extends past the end of dst")
    pt = (np.full(n, CRC_INITIAL_REGISTER, dtype=np.uint64) if partials is None
          else np.asarray(partials, dtype=np.uint64) & 0xFFFFFFFF)
    host = np.empty((n, 4), dtype=np.uint64)
    host[:, 0] = np.uint64(src.data_ptr()) + so
    host[:, 1] = np.uint64(dst.data_ptr()) + do
    host[:, 2] = cl | (sl << np.uint64(32))
    host[:, 3] = pt
    return torch.from_numpy(host.view(np.int64)).to(src.device)


def frag_bcopy_batch(descs: torch.Tensor, n: int | None = None, mode: int = CRC32, out: torch.Tensor | None = None,
                     stream: torch.cuda.Stream | None = None, rows_hint: int = 0) -> torch.Tensor:
    """Fused bcopy_uicrc / bcopy_uicsum per ``lampi_copy_desc``; returns the checksums.
    rows_hint: LAMPI_CSUM_ROWS_HINT -- fragments span about that many 4 KiB rows (row groups)."""
    _require_cuda(descs, "descs")
    count = descs.numel() * descs.element_size() // 32 if n is None else int(n)
    if mode == NONE:  # checksumming off: copies only, no output (returns None)
        check(lib().lampi_frag_bcopy_batch(descs.data_ptr(), count, None, mode | rows_hint_bits(rows_hint),
                                           _stream_handle(stream)), "lampi_frag_bcopy_batch")
        return None
    if out is None:
        out = torch.empty(count, dtype=torch.int32, device=descs.device)
    _require_cuda(out, "out")
    if out.numel() < count:
        raise ValueError("out is too small")
    check(lib().lampi_frag_bcopy_batch(descs.data_ptr(), count, out.data_ptr(), mode | rows_hint_bits(rows_hint),
                                       _stream_handle(stream)),
          "lampi_frag_bcopy_batch")
    return out


def _strided_dst(dst: torch.Tensor | None, count: int, stride: int, offset: int, mode: int) -> int | None:
    """Device address of record 0's output word (None with mode NONE: nothing is written)."""
    if mode == NONE:
        return None
    if dst is None:
        raise ValueError("dst is required unless mode is NONE")
    _records(dst.view(torch.uint8)[offset:], count, stride, "dst")
    return dst.data_ptr() + offset


def frag_bcopy_batch_strided(descs: torch.Tensor, dst: torch.Tensor | None, stride: int, offset: int = 0,
                             n: int | None = None, mode: int = CRC32, stream: torch.cuda.Stream | None = None,
                             rows_hint: int = 0) -> torch.Tensor | None:
    """frag_bcopy_batch with checksum i written at byte offset + i*stride of ``dst`` (e.g. dataChecksum @64
    of each buffer of a GM send ring, src/path/gm/sendFrag.cc:149-151); returns ``dst``."""
    _require_cuda(descs, "descs")
    count = descs.numel() * descs.element_size() // 32 if n is None else int(n)
    ptr = _strided_dst(dst, count, stride, offset, mode)
    check(lib().lampi_frag_bcopy_batch_strided(descs.data_ptr(), count, ptr, stride, mode | rows_hint_bits(rows_hint),
                                               _stream_handle(stream)), "lampi_frag_bcopy_batch_strided")
    return dst


def frag_csum_batch(descs: torch.Tensor, n: int | None = None, mode: int = CRC32, out: torch.Tensor | None = None,
                    stream: torch.cuda.Stream | None = None, by_bytes: bool = False, rows_hint: int = 0) -> torch.Tensor:
    """out[i] = checksum of fragment descs[i] (piece streams: fragments of any size share rows).
    by_bytes: LAMPI_CSUM_BY_BYTES -- plan the work by bytes (large fragments split across workgroups).
    rows_hint: LAMPI_CSUM_ROWS_HINT -- fragments span about that many 4 KiB rows: each runs as that many
    row segments computed on the device (no plan launch)."""
    _require_cuda(descs, "descs")
    count = descs.numel() * descs.element_size() // 16 if n is None else int(n)
    if out is None:
        out = torch.empty(count, dtype=torch.int32, device=descs.device)
    _require_cuda(out, "out")
    if out.numel() < count:
        raise ValueError("out is too small")
    check(lib().lampi_frag_csum_batch(descs.data_ptr(), count, out.data_ptr(),
                                      mode | (BY_BYTES if by_bytes else 0) | rows_hint_bits(rows_hint),
                                      _stream_handle(stream)), "lampi_frag_csum_batch")
    return out


def diag_frag_csum_batch_per_wave(descs: torch.Tensor, n: int | None = None, mode: int = CRC32,
                                  out: torch.Tensor | None = None,
                                  stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """lampi_frag_csum_batch's results on the one-wavefront-per-fragment schedule: the internal diagnostic
    lampi_diag_frag_csum_batch_per_wave (not part of include/lampi_csum.h since round 5; bench.py's config C
    comparison and the parity tests)."""
    import ctypes

    fn = lib().lampi_diag_frag_csum_batch_per_wave
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    _require_cuda(descs, "descs")
    count = descs.numel() * descs.element_size() // 16 if n is None else int(n)
    if out is None:
        out = torch.empty(count, dtype=torch.int32, device=descs.device)
    _require_cuda(out, "out")
    if out.numel() < count:
        raise ValueError("out is too small")
    check(fn(descs.data_ptr(), count, out.data_ptr(), mode, _stream_handle(stream)),
          "lampi_diag_frag_csum_batch_per_wave")
    return out


def frag_csum_batch_strided(descs: torch.Tensor, dst: torch.Tensor, stride: int, offset: int = 0,
                            n: int | None = None, mode: int = CRC32,
                            stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """Checksum i of the batch written at byte offset + i*stride of ``dst`` (e.g. the
    dataChecksum field, offset 64, of 72-byte gmHeaderData records); returns ``dst``."""
    _require_cuda(descs, "descs")
    count = descs.numel() * descs.element_size() // 16 if n is None else int(n)
    _records(dst[offset:] if dst.element_size() == 1 else dst.view(torch.uint8)[offset:], count, stride, "dst")
    check(lib().lampi_frag_csum_batch_strided(descs.data_ptr(), count, dst.data_ptr() + offset, stride, mode,
                                              _stream_handle(stream)), "lampi_frag_csum_batch_strided")
    return dst


def frag_csum64_batch(descs: torch.Tensor, n: int | None = None, out: torch.Tensor | None = None,
                      stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """out[i] = 64-bit csum (fresh state) of fragment descs[i] (int64 storage, read as uint64)."""
    _require_cuda(descs, "descs")
    count = descs.numel() * descs.element_size() // 16 if n is None else int(n)
    if out is None:
        out = torch.empty(count, dtype=torch.int64, device=descs.device)
    _require_cuda(out, "out")
    if out.numel() * out.element_size() < 8 * count:
        raise ValueError("out is too small")
    check(lib().lampi_frag_csum64_batch(descs.data_ptr(), count, out.data_ptr(), _stream_handle(stream)),
          "lampi_frag_csum64_batch")
    return out


def msg_csum(msg: torch.Tensor, frag_len: int, partial: int = CRC_INITIAL_REGISTER, mode: int = CRC32,
             msg_len: int | None = None, out: torch.Tensor | None = None,
             stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """Checksums of the fragments of a contiguous device message (src/path/gm/path.cc:98-121)."""
    _require_cuda(msg, "msg")
    nbytes = msg.numel() * msg.element_size() if msg_len is None else int(msg_len)
    if nbytes > msg.numel() * msg.element_size():
        raise ValueError("msg_len exceeds the tensor")
    n = (nbytes + frag_len - 1) // frag_len if nbytes else 1
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=msg.device)
    _require_cuda(out, "out")
    if out.numel() < n:
        raise ValueError("out is too small")
    check(lib().lampi_msg_csum(msg.data_ptr(), nbytes, frag_len, partial & 0xFFFFFFFF, out.data_ptr(), mode,
                               _stream_handle(stream)), "lampi_msg_csum")
    return out


def msg_bcopy(msg: torch.Tensor, frag_len: int, dst: torch.Tensor, dst_stride: int | None = None,
              partial: int = CRC_INITIAL_REGISTER, mode: int = CRC32, msg_len: int | None = None,
              out: torch.Tensor | None = None, stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """Fragment ``msg`` and copy fragment k to ``dst`` + k*dst_stride with its checksum fused."""
    _require_cuda(msg, "msg")
    _require_cuda(dst, "dst")
    nbytes = msg.numel() * msg.element_size() if msg_len is None else int(msg_len)
    if nbytes > msg.numel() * msg.element_size():
        raise ValueError("msg_len exceeds the tensor")
    stride = frag_len if dst_stride is None else int(dst_stride)
    n = (nbytes + frag_len - 1) // frag_len if nbytes else 1
    if nbytes and (n - 1) * stride + (nbytes - (n - 1) * frag_len) > dst.numel() * dst.element_size():
        raise ValueError("dst is too small")
    if mode == NONE:  # checksumming off: copies only (returns None)
        check(lib().lampi_msg_bcopy(msg.data_ptr(), nbytes, frag_len, dst.data_ptr(), stride, partial & 0xFFFFFFFF,
                                    None, mode, _stream_handle(stream)), "lampi_msg_bcopy")
        return None
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=msg.device)
    _require_cuda(out, "out")
    if out.numel() < n:
        raise ValueError("out is too small")
    check(lib().lampi_msg_bcopy(msg.data_ptr(), nbytes, frag_len, dst.data_ptr(), stride, partial & 0xFFFFFFFF,
                                out.data_ptr(), mode, _stream_handle(stream)), "lampi_msg_bcopy")
    return out


def msg_bcopy_strided(msg: torch.Tensor, frag_len: int, dst: torch.Tensor, dst_stride: int, out: torch.Tensor | None,
                      out_stride: int, out_offset: int = 0, partial: int = CRC_INITIAL_REGISTER, mode: int = CRC32,
                      msg_len: int | None = None, stream: torch.cuda.Stream | None = None) -> None:
    """msg_bcopy with fragment k's checksum written at byte out_offset + k*out_stride of ``out``: a GM send into
    a ring of header + payload buffers (dst = ring[72:], out = ring, out_offset 64, both strides the buffer size)."""
    _require_cuda(msg, "msg")
    _require_cuda(dst, "dst")
    nbytes = msg.numel() * msg.element_size() if msg_len is None else int(msg_len)
    if nbytes > msg.numel() * msg.element_size():
        raise ValueError("msg_len exceeds the tensor")
    n = (nbytes + frag_len - 1) // frag_len if nbytes else 1
    if nbytes and (n - 1) * dst_stride + (nbytes - (n - 1) * frag_len) > dst.numel() * dst.element_size():
        raise ValueError("dst is too small")
    ptr = _strided_dst(out, n, out_stride, out_offset, mode)
    check(lib().lampi_msg_bcopy_strided(msg.data_ptr(), nbytes, frag_len, dst.data_ptr(), dst_stride,
                                        partial & 0xFFFFFFFF, ptr, out_stride, mode, _stream_handle(stream)),
          "lampi_msg_bcopy_strided")


def chain_csum_batch(pieces: torch.Tensor, first, mode: int = CRC32, out: torch.Tensor | None = None,
                     stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """Chained checksum per fragment over its typemap pieces (``lampi_copy_desc`` rows of
    ``pieces``; fragment f = pieces first[f] .. first[f+1]-1)."""
    _require_cuda(pieces, "pieces")
    npieces = pieces.numel() * pieces.element_size() // 32
    fa = np.asarray(first, dtype=np.uint32) if not isinstance(first, torch.Tensor) else None
    if fa is not None:
        if fa.size < 1 or (fa.size > 1 and (np.any(np.diff(fa.astype(np.int64)) < 0) or int(fa[-1]) > npieces)):
            raise ValueError("first must be nondecreasing and end at most at the piece count")
        first_t = torch.from_numpy(fa.view(np.int32)).to(pieces.device)
    else:
        _require_cuda(first, "first")
        first_t = first
    nfrags = first_t.numel() - 1
    if mode == NONE:  # checksumming off: the pieces are copied, no output (returns None)
        check(lib().lampi_chain_csum_batch(pieces.data_ptr(), npieces, first_t.data_ptr(), nfrags, None, mode,
                                           _stream_handle(stream)), "lampi_chain_csum_batch")
        return None
    if out is None:
        out = torch.empty(max(nfrags, 0), dtype=torch.int32, device=pieces.device)
    check(lib().lampi_chain_csum_batch(pieces.data_ptr(), npieces, first_t.data_ptr(), nfrags, out.data_ptr(), mode,
                                       _stream_handle(stream)), "lampi_chain_csum_batch")
    return out


def chain_csum_batch_strided(pieces: torch.Tensor, first: torch.Tensor, dst: torch.Tensor | None, stride: int,
                             offset: int = 0, mode: int = CRC32, stream: torch.cuda.Stream | None = None):
    """chain_csum_batch with fragment f's checksum written at byte offset + f*stride of ``dst`` (the typemap
    send's dataChecksum, src/path/gm/sendFrag.cc:216); ``first`` a device int32 tensor of nfrags + 1 offsets."""
    _require_cuda(pieces, "pieces")
    _require_cuda(first, "first")
    npieces = pieces.numel() * pieces.element_size() // 32
    nfrags = first.numel() - 1
    ptr = _strided_dst(dst, nfrags, stride, offset, mode)
    check(lib().lampi_chain_csum_batch_strided(pieces.data_ptr(), npieces, first.data_ptr(), nfrags, ptr, stride,
                                               mode, _stream_handle(stream)), "lampi_chain_csum_batch_strided")
    return dst


def chain_copy_to_app_batch(pieces: torch.Tensor, first, expected: torch.Tensor | None, expected_stride: int = 4,
                            mode: int = CRC32, stream: torch.cuda.Stream | None = None):
    """RecvDesc_t::CopyToApp's non-contiguous branch (src/path/common/BaseDesc.cc:326-340): the typemap
    pieces of each received fragment copied, the checksum from CRC_INITIAL_REGISTER compared with
    expected (None with mode NONE).  Returns (copied int64 -- len_copied or -1 --, csum int32, mask, nbad)."""
    _require_cuda(pieces, "pieces")
    npieces = pieces.numel() * pieces.element_size() // 32
    fa = np.asarray(first, dtype=np.uint32) if not isinstance(first, torch.Tensor) else None
    if fa is not None:
        if fa.size < 1 or (fa.size > 1 and (np.any(np.diff(fa.astype(np.int64)) < 0) or int(fa[-1]) > npieces)):
            raise ValueError("first must be nondecreasing and end at most at the piece count")
        first_t = torch.from_numpy(fa.view(np.int32)).to(pieces.device)
    else:
        _require_cuda(first, "first")
        first_t = first
    nfrags = first_t.numel() - 1
    if expected is not None:
        _records(expected, nfrags, expected_stride, "expected")
    copied = torch.empty(max(nfrags, 1), dtype=torch.int64, device=pieces.device)
    csum = torch.empty(max(nfrags, 1), dtype=torch.int32, device=pieces.device)
    mask = torch.empty(max((nfrags + 31) // 32, 1), dtype=torch.int32, device=pieces.device)
    nbad = torch.empty(1, dtype=torch.int32, device=pieces.device)
    check(lib().lampi_chain_copy_to_app_batch(pieces.data_ptr(), npieces, first_t.data_ptr(), nfrags,
                                              0 if expected is None else expected.data_ptr(), expected_stride,
                                              copied.data_ptr(), csum.data_ptr(), mask.data_ptr(), nbad.data_ptr(),
                                              mode, _stream_handle(stream)), "lampi_chain_copy_to_app_batch")
    return copied[:nfrags], csum[:nfrags], mask, nbad


def _records(t: torch.Tensor, n: int, stride: int, what: str) -> None:
    _require_cuda(t, what)
    if n and (n - 1) * stride + 4 > t.numel() * t.element_size():
        raise ValueError(f"{what} is too small for {n} records of stride {stride}")


def header_csum_batch(hdrs: torch.Tensor, n: int, stride: int, crclen: int, word_count: int, mode: int = CRC32,
                      out: torch.Tensor | None = None, stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """BasePath_t::headerChecksum of n headers ``stride`` bytes apart (src/path/common/path.h:280-314)."""
    _records(hdrs, n, stride, "hdrs")
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=hdrs.device)
    check(lib().lampi_header_csum_batch(hdrs.data_ptr(), n, stride, crclen, word_count, out.data_ptr(), mode,
                                        _stream_handle(stream)), "lampi_header_csum_batch")
    return out


def header_csum_batch_strided(hdrs: torch.Tensor, n: int, stride: int, crclen: int, word_count: int,
                              dst: torch.Tensor, out_stride: int, offset: int = 0, mode: int = CRC32,
                              stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """headerChecksum of n headers written at byte offset + i*out_stride of ``dst``: in place into the headers
    with dst = hdrs, offset 68, out_stride = stride (src/path/gm/sendFrag.cc:218-225); mode NONE writes nothing."""
    _records(hdrs, n, stride, "hdrs")
    ptr = _strided_dst(dst, n, out_stride, offset, mode)
    check(lib().lampi_header_csum_batch_strided(hdrs.data_ptr(), n, stride, crclen, word_count, ptr, out_stride, mode,
                                                _stream_handle(stream)), "lampi_header_csum_batch_strided")
    return dst


def _mask_out(n: int, device) -> tuple[torch.Tensor, torch.Tensor]:
    return (torch.zeros(max(1, (n + 31) // 32), dtype=torch.int32, device=device),
            torch.zeros(1, dtype=torch.int32, device=device))


def header_check_batch(hdrs: torch.Tensor, n: int, stride: int, hdr_bytes: int, word_count: int, csum_offset: int,
                       mode: int = CRC32, stream: torch.cuda.Stream | None = None):
    """Receiver header check (src/path/gm/path.cc:364-393); returns (mask, nbad), mask bit set = bad."""
    _records(hdrs, n, stride, "hdrs")
    mask, nbad = _mask_out(n, hdrs.device)
    check(lib().lampi_header_check_batch(hdrs.data_ptr(), n, stride, hdr_bytes, word_count, csum_offset,
                                         mask.data_ptr(), nbad.data_ptr(), mode, _stream_handle(stream)),
          "lampi_header_check_batch")
    return mask, nbad


def header_compare_batch(hdrs: torch.Tensor, n: int, stride: int, crclen: int, csum_offset: int, mode: int = CRC32,
                         stream: torch.cuda.Stream | None = None):
    """The IB receiver's header check (src/path/ib/path.cc:652-680): uicrc / uicsum of crclen bytes vs the
    stored, unswapped word at csum_offset; returns (mask, nbad), mask bit set = bad."""
    _records(hdrs, n, stride, "hdrs")
    mask, nbad = _mask_out(n, hdrs.device)
    check(lib().lampi_header_compare_batch(hdrs.data_ptr(), n, stride, crclen, csum_offset, mask.data_ptr(),
                                           nbad.data_ptr(), mode, _stream_handle(stream)),
          "lampi_header_compare_batch")
    return mask, nbad


def check_data_batch(calc: torch.Tensor, expected: torch.Tensor, expected_stride: int = 4,
                     lengths: torch.Tensor | None = None, lengths_stride: int = 4, n: int | None = None,
                     expected_offset: int = 0, lengths_offset: int = 0, stream: torch.cuda.Stream | None = None):
    """CheckData over a batch (src/path/gm/recvFrag.h:213-257); returns (mask, nbad), bit set = corrupt."""
    _require_cuda(calc, "calc")
    count = calc.numel() if n is None else int(n)
    _records(expected, count, expected_stride, "expected")
    lp = 0
    if lengths is not None:
        _records(lengths, count, lengths_stride, "lengths")
        lp = lengths.data_ptr() + lengths_offset
    mask, nbad = _mask_out(count, calc.device)
    check(lib().lampi_check_data_batch(calc.data_ptr(), expected.data_ptr() + expected_offset, expected_stride,
                                       lp or None, lengths_stride, count, mask.data_ptr(), nbad.data_ptr(),
                                       _stream_handle(stream)), "lampi_check_data_batch")
    return mask, nbad


def make_recv_descs(frag: torch.Tensor, frag_offsets, app: torch.Tensor, app_offsets, lengths,
                    app_lens) -> torch.Tensor:
    """Build a device array of ``lampi_recv_desc`` (n x 32 bytes, int64 [n, 4] storage): fragment i
    = ``lengths[i]`` received bytes at frag + frag_offsets[i], delivered to app + app_offsets[i]
    with ``app_lens[i]`` bytes of room left in the posted buffer (posted length - offset, may be
    <= 0; ref src/path/common/BaseDesc.cc:300-307)."""
    _require_cuda(frag, "frag")
    _require_cuda(app, "app")
    fo = np.asarray(frag_offsets, dtype=np.uint64)
    ao = np.asarray(app_offsets, dtype=np.uint64)
    ln = np.asarray(lengths, dtype=np.uint64)
    al = np.asarray(app_lens, dtype=np.int64)
    n = fo.size
    if not (ao.size == ln.size == al.size == n):
        raise ValueError("descriptor fields differ in size")
    if n:
        if int(ln.max()) > 0xFFFFFFFF:
            raise ValueError("fragment length exceeds 32 bits")
        if int((fo + ln).max()) > frag.numel() * frag.element_size():
            raise ValueError("a fragment extends past the end of frag")
        copy = np.minimum(ln.astype(np.int64), np.maximum(al, 0))
        if int((ao.astype(np.int64) + copy).max()) > app.numel() * app.element_size():
            raise ValueError("a delivery extends past the end of app")
    host = np.empty((n, 4), dtype=np.uint64)
    host[:, 0] = np.uint64(frag.data_ptr()) + fo
    host[:, 1] = np.uint64(app.data_ptr()) + ao
    host[:, 2] = al.view(np.uint64)
    host[:, 3] = ln
    return torch.from_numpy(host.view(np.int64)).to(frag.device)


def copy_to_app_batch(descs: torch.Tensor, expected: torch.Tensor, expected_stride: int = 4, expected_offset: int = 0,
                      n: int | None = None, mode: int = CRC32, stream: torch.cuda.Stream | None = None,
                      rows_hint: int = 0):
    """RecvDesc_t::CopyToApp over a batch (src/path/common/BaseDesc.cc:288-342): returns
    (copied int64[n] -- bytes copied or -1 when corrupt --, csum int32[n], mask, nbad).
    rows_hint: as for frag_bcopy_batch (GM's 65,456-byte payloads: 16)."""
    _require_cuda(descs, "descs")
    count = descs.numel() * descs.element_size() // 32 if n is None else int(n)
    if expected is None:  # (mode NONE: nothing compared; the C call refuses a null pointer in the other modes)
        if (mode & 0xFF) != NONE:
            raise ValueError("expected is required unless mode is NONE (checksumming off)")
        exp_ptr, expected_stride = 0, 0
    else:
        _records(expected.view(torch.uint8)[expected_offset:] if count else expected, count, expected_stride,
                 "expected")
        exp_ptr = expected.data_ptr() + expected_offset
    copied = torch.empty(max(count, 1), dtype=torch.int64, device=descs.device)
    csum = torch.empty(max(count, 1), dtype=torch.int32, device=descs.device)
    # (the call zeroes the mask words and the count itself: no fill kernels here, except for an empty batch)
    mask, nbad = (_mask_out(count, descs.device) if count == 0 else
                  (torch.empty((count + 31) // 32, dtype=torch.int32, device=descs.device),
                   torch.empty(1, dtype=torch.int32, device=descs.device)))
    check(lib().lampi_copy_to_app_batch(descs.data_ptr(), count, exp_ptr or None, expected_stride,
                                        copied.data_ptr(), csum.data_ptr(), mask.data_ptr(), nbad.data_ptr(),
                                        mode | rows_hint_bits(rows_hint), _stream_handle(stream)),
          "lampi_copy_to_app_batch")
    return copied[:count], csum[:count], mask, nbad


def mask_bits(mask: torch.Tensor, n: int) -> np.ndarray:
    """Device mask words -> bool array of length n (True = failed)."""
    w = mask.cpu().numpy().view(np.uint32)
    return ((w[np.arange(n) // 32] >> (np.arange(n) % 32).astype(np.uint32)) & 1).astype(bool)


def fill_stream(dst: torch.Tensor, seed: int, byte_off: int = 0, nbytes: int | None = None,
                stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """Write the SURVEY.md 8(d) synthetic stream (splitmix64 words, LE) into ``dst`` on device."""
    _require_cuda(dst, "dst")
    n = dst.numel() * dst.element_size() if nbytes is None else int(nbytes)
    check(lib().lampi_fill_stream(dst.data_ptr(), n, seed & (2**64 - 1), byte_off, _stream_handle(stream)),
          "lampi_fill_stream")
    return dst


def fill_stream_frags(dst: torch.Tensor, n: int, frag_len: int, seed: int, k0: int = 0, kstep: int = 1,
                      stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """Round-robin shard of a global batch: fragment i of ``dst`` = global fragment k0 + i*kstep."""
    _require_cuda(dst, "dst")
    if n * frag_len > dst.numel() * dst.element_size():
        raise ValueError("dst is too small")
    check(lib().lampi_fill_stream_frags(dst.data_ptr(), n, frag_len, seed & (2**64 - 1), k0, kstep,
                                        _stream_handle(stream)), "lampi_fill_stream_frags")
    return dst
