"""oracle.py -- ctypes access to the TEST-ONLY checkers.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product (lampi_amd/).

* :class:`Restatement` -- oracle/libcsum_ref.so, the clean-room C restatement (csum_ref.c).
  Travels to the GPU box; it is the parity checker there and the timed CPU baseline.
* :class:`Reference` -- oracle/_ref/libref_memfunctions.so, the reference's own
  src/util/MemFunctions.cc compiled unmodified (oracle/Makefile).  Exists only where
  /root/reference was present at build time; bound by the C++ mangled names of
  SURVEY.md 8(b).

Parity status: pinned (tests/golden/ fixtures generated from Reference, checked against
Restatement by tests/test_oracle.py).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
RESTATEMENT_SO = os.path.join(HERE, "libcsum_ref.so")
REFERENCE_SO = os.path.join(HERE, "_ref", "libref_memfunctions.so")

CRC_INIT = 0xFFFFFFFF
_u = ctypes.c_uint
_ul = ctypes.c_ulong
_vp = ctypes.c_void_p
_pu = ctypes.POINTER(ctypes.c_uint)
_pul = ctypes.POINTER(ctypes.c_ulong)


def _buf(b):
    arr = np.frombuffer(b, dtype=np.uint8) if not isinstance(b, np.ndarray) else b.view(np.uint8).reshape(-1)
    return arr.ctypes.data, arr


class _Api:
    """Common Python surface: uicrc / bcopy_uicrc / uicsum / bcopy_uicsum."""

    def uicrc(self, data, n=None, partial=CRC_INIT):
        p, a = _buf(data)
        return int(self._uicrc(p, a.size if n is None else n, partial & 0xFFFFFFFF))

    def bcopy_uicrc(self, src, dst, copylen, crclen, partial=CRC_INIT):
        ps, _ = _buf(src)
        pd, _ = _buf(dst)
        return int(self._bcopy_uicrc(ps, pd, copylen, crclen, partial & 0xFFFFFFFF))

    def uicsum(self, data, n=None, pint=0, plen=0):
        """Returns (sum_increment, pint', plen')."""
        p, a = _buf(data)
        pi, pl = _u(pint), _u(plen)
        r = self._uicsum(p, a.size if n is None else n, ctypes.byref(pi), ctypes.byref(pl))
        return int(r), pi.value, pl.value

    def bcopy_uicsum(self, src, dst, copylen, csumlen, pint=0, plen=0):
        ps, _ = _buf(src)
        pd, _ = _buf(dst)
        pi, pl = _u(pint), _u(plen)
        r = self._bcopy_uicsum(ps, pd, copylen, csumlen, ctypes.byref(pi), ctypes.byref(pl))
        return int(r), pi.value, pl.value

    def csum(self, data, n=None, plong=0, plen=0):
        """64-bit csum: returns (sum_increment, plong', plen')."""
        p, a = _buf(data)
        pi, pl = _ul(plong), _ul(plen)
        r = self._csum(p, a.size if n is None else n, ctypes.byref(pi), ctypes.byref(pl))
        return int(r), pi.value, pl.value

    def bcopy_csum(self, src, dst, copylen, csumlen, plong=0, plen=0):
        ps, _ = _buf(src)
        pd, _ = _buf(dst)
        pi, pl = _ul(plong), _ul(plen)
        r = self._bcopy_csum(ps, pd, copylen, csumlen, ctypes.byref(pi), ctypes.byref(pl))
        return int(r), pi.value, pl.value


def copy_to_app(api: "_Api", frag: np.ndarray, length: int, app_len: int, expected: int, usecrc: bool):
    """RecvDesc_t::CopyToApp for one contiguous fragment (ref src/path/common/BaseDesc.cc:288-342)
    with the GM hooks CopyFunction (src/path/gm/recvFrag.h:165-182) and CheckData (:213-257),
    checksumming on: lengthToCopy = min(length_m, AppBufferLen); AppBufferLen <= 0 is DataOK with
    nothing copied; otherwise bcopy_uicrc / bcopy_uicsum(frag, app, lengthToCopy, length_m)
    (CRC_INITIAL_REGISTER or 0 for a zero lengthToCopy) and CheckData(csum, lengthToCopy).
    Returns (CopyToApp's return value -- bytes or -1 --, the checksum CopyFunction returned (the
    CopyFunction-of-nothing value when it is not called), the bytes delivered)."""
    empty = CRC_INIT if usecrc else 0
    if app_len <= 0:
        return 0, empty, np.zeros(0, np.uint8)
    n = min(length, app_len)
    dst = np.zeros(n, np.uint8)
    if n == 0:
        return 0, empty, dst
    c = api.bcopy_uicrc(frag, dst, n, length) if usecrc else api.bcopy_uicsum(frag, dst, n, length)[0]
    return (n if c == expected else -1), c, dst


def copy_to_app_nochecksum(frag: np.ndarray, length: int, app_len: int):
    """RecvDesc_t::CopyToApp (ref src/path/common/BaseDesc.cc:288-342) with checksumming off
    (gmState.doChecksum == false, src/path/gm/state.h:140; mpirun -mf nochecksum, src/run/Input.cc:1986-2067):
    CopyFunction only copies lengthToCopy bytes and returns 0 (src/path/gm/recvFrag.h:178-181), CheckData passes
    (:231-232).  Returns (bytes copied, 0 -- the checksum output the batch defines --, the bytes delivered)."""
    if app_len <= 0:
        return 0, 0, np.zeros(0, np.uint8)
    n = min(length, app_len)
    return n, 0, np.array(frag[:n], np.uint8)


def non_contiguous_copy_to_app(api: "_Api", pieces: list, expected: int, mode: int):
    """CopyToApp's non-contiguous branch (ref src/path/common/BaseDesc.cc:326-340): non_contiguous_copy
    (:72-163) calls nonContigCopyFunction once per typemap piece (GM src/path/gm/recvFrag.h:186-211) -- CRC:
    the register from CRC_INITIAL_REGISTER on the first call, bcopy_uicrc(piece, len, len, register); SUM:
    *checkSum = 0 (:124-125), += bcopy_uicsum with the partial-word state threaded; checksumming off: memcpy
    only -- then CheckData(checkSum, len_copied) (gm/recvFrag.h:213-257).  pieces: the pieces' source bytes
    in order; mode 0 CRC, 1 SUM, 2 off.  Returns (len_copied or -1, the checksum)."""
    copied = int(sum(int(p.size) for p in pieces))
    if mode == 2:
        return copied, 0
    if mode == 0:
        c = CRC_INIT
        for p in pieces:
            c = api.bcopy_uicrc(p, np.zeros(max(p.size, 1), np.uint8), p.size, p.size, c)
    else:
        c, pi, pl = 0, 0, 0
        for p in pieces:
            r, pi, pl = api.bcopy_uicsum(p, np.zeros(max(p.size, 1), np.uint8), p.size, p.size, pi, pl)
            c = (c + r) & 0xFFFFFFFF
    ok = copied == 0 or c == expected
    return (copied if ok else -1), c


class Restatement(_Api):
    def __init__(self, path: str = RESTATEMENT_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        L = ctypes.CDLL(path)
        self.lib = L
        self._uicrc = L.oracle_uicrc
        self._uicrc.restype, self._uicrc.argtypes = _u, [_vp, ctypes.c_size_t, _u]
        self._bcopy_uicrc = L.oracle_bcopy_uicrc
        self._bcopy_uicrc.restype = _u
        self._bcopy_uicrc.argtypes = [_vp, _vp, ctypes.c_size_t, ctypes.c_size_t, _u]
        self._uicsum = L.oracle_uicsum
        self._uicsum.restype, self._uicsum.argtypes = _u, [_vp, ctypes.c_size_t, _pu, _pu]
        self._bcopy_uicsum = L.oracle_bcopy_uicsum
        self._bcopy_uicsum.restype = _u
        self._bcopy_uicsum.argtypes = [_vp, _vp, ctypes.c_size_t, ctypes.c_size_t, _pu, _pu]
        self._csum = L.oracle_csum64
        self._csum.restype, self._csum.argtypes = ctypes.c_uint64, [_vp, ctypes.c_size_t, _pul, _pul]
        self._bcopy_csum = L.oracle_bcopy_csum64
        self._bcopy_csum.restype = ctypes.c_uint64
        self._bcopy_csum.argtypes = [_vp, _vp, ctypes.c_size_t, ctypes.c_size_t, _pul, _pul]
        L.oracle_fill_stream.argtypes = [_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t]
        L.oracle_uniform_batch.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_size_t,
                                           ctypes.c_int, ctypes.c_int, _vp]
        L.oracle_uniform_digest.argtypes = [ctypes.c_uint64, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp]
        L.oracle_desc_batch.argtypes = [_vp, _vp, _vp, _vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, _vp]
        L.oracle_time_uniform.restype = ctypes.c_double
        L.oracle_time_uniform.argtypes = [ctypes.c_uint64, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                                          ctypes.c_int, _vp]
        L.oracle_time_fn.restype = ctypes.c_double
        L.oracle_time_fn.argtypes = [_vp, _vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, _vp, _vp]
        L.oracle_zipf_lengths.restype = ctypes.c_size_t
        L.oracle_zipf_lengths.argtypes = [ctypes.c_uint64, ctypes.c_size_t, _vp]
        L.oracle_header_checksum.restype = _u
        L.oracle_header_checksum.argtypes = [_vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int]

    # ---- batch helpers -------------------------------------------------------------
    def stream(self, seed: int, byte_off: int, n: int) -> np.ndarray:
        out = np.empty(n, dtype=np.uint8)
        self.lib.oracle_fill_stream(out.ctypes.data, seed, byte_off, n)
        return out

    def uniform_batch(self, seed: int, k0: int, n: int, L: int, mode: int, nthreads: int = 0) -> np.ndarray:
        out = np.empty(n, dtype=np.uint32)
        self.lib.oracle_uniform_batch(seed, k0, n, L, mode, nthreads, out.ctypes.data)
        return out

    def uniform_digest(self, seed: int, n: int, L: int, mode: int, nshard: int = 1, shard: int = 0,
                       nthreads: int = 0) -> tuple[int, int]:
        dig = np.zeros(2, dtype=np.uint32)
        self.lib.oracle_uniform_digest(seed, n, L, mode, nshard, shard, nthreads, dig.ctypes.data)
        return int(dig[0]), int(dig[1])

    def desc_batch(self, base: np.ndarray, offsets, lengths, partials=None, mode: int = 0,
                   nthreads: int = 0) -> np.ndarray:
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        pt = None if partials is None else np.ascontiguousarray(partials, dtype=np.uint32)
        out = np.empty(off.size, dtype=np.uint32)
        self.lib.oracle_desc_batch(base.ctypes.data, off.ctypes.data, ln.ctypes.data,
                                   None if pt is None else pt.ctypes.data, off.size, mode, nthreads,
                                   out.ctypes.data)
        return out

    def time_uniform(self, seed: int, n: int, L: int, mode: int, nthreads: int) -> tuple[float, int]:
        x = ctypes.c_uint(0)
        t = self.lib.oracle_time_uniform(seed, n, L, mode, nthreads, ctypes.byref(x))
        return float(t), x.value

    def time_crc_fn(self, fn_addr: int, buf: np.ndarray, n: int, L: int, nthreads: int,
                    out: np.ndarray | None = None) -> tuple[float, int]:
        """Seconds for `fn` (uicrc-shaped C function address) over n fragments of L bytes;
        the per-fragment values land in `out` (u32[n]) when given."""
        x = ctypes.c_uint(0)
        if out is not None and (out.dtype != np.uint32 or out.size < n or not out.flags.c_contiguous):
            raise ValueError("out must be a contiguous u32 array of n values")
        t = self.lib.oracle_time_fn(fn_addr, buf.ctypes.data, n, L, nthreads, ctypes.byref(x),
                                    None if out is None else out.ctypes.data)
        return float(t), x.value

    def uicrc_addr(self) -> int:
        return ctypes.cast(self.lib.oracle_uicrc, ctypes.c_void_p).value

    def zipf_lengths(self, min_total: int) -> np.ndarray:
        """Config C fragment lengths, packed until the total >= min_total."""
        n = int(self.lib.oracle_zipf_lengths(min_total, 0, None))
        out = np.empty(n, dtype=np.uint32)
        self.lib.oracle_zipf_lengths(min_total, n, out.ctypes.data)
        return out

    def header_checksum(self, hdr, crclen: int, word_count: int, usecrc: bool) -> int:
        p, _ = _buf(hdr)
        return int(self.lib.oracle_header_checksum(p, crclen, word_count, 1 if usecrc else 0))


class Reference(_Api):
    """The reference's MemFunctions.cc, compiled unmodified (C++ linkage, mangled names)."""

    def uicrc_addr(self) -> int:
        return ctypes.cast(self._uicrc, ctypes.c_void_p).value

    def __init__(self, path: str = REFERENCE_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing (built only where /root/reference exists)")
        L = ctypes.CDLL(path)
        self.lib = L
        self._uicrc = getattr(L, "_Z5uicrcPKvmj")
        self._uicrc.restype, self._uicrc.argtypes = _u, [_vp, _ul, _u]
        self._bcopy_uicrc = getattr(L, "_Z11bcopy_uicrcPKvPvmmj")
        self._bcopy_uicrc.restype, self._bcopy_uicrc.argtypes = _u, [_vp, _vp, _ul, _ul, _u]
        self._uicsum = getattr(L, "_Z6uicsumPKvmPjS1_")
        self._uicsum.restype, self._uicsum.argtypes = _u, [_vp, _ul, _pu, _pu]
        self._bcopy_uicsum = getattr(L, "_Z12bcopy_uicsumPKvPvmmPjS2_")
        self._bcopy_uicsum.restype, self._bcopy_uicsum.argtypes = _u, [_vp, _vp, _ul, _ul, _pu, _pu]
        self._csum = getattr(L, "_Z4csumPKvmPmS1_")
        self._csum.restype, self._csum.argtypes = _ul, [_vp, _ul, _pul, _pul]
        self._bcopy_csum = getattr(L, "_Z10bcopy_csumPKvPvmmPmS2_")
        self._bcopy_csum.restype, self._bcopy_csum.argtypes = _ul, [_vp, _vp, _ul, _ul, _pul, _pul]


def splitmix_stream(seed: int, byte_off: int, n: int) -> np.ndarray:
    """numpy generator of the SURVEY.md 8(d) stream (same bytes as oracle_fill_stream)."""
    w0 = byte_off // 8
    w1 = (byte_off + n + 7) // 8
    idx = np.arange(w0, w1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (idx + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z ^= z >> np.uint64(30)
        z *= np.uint64(0xBF58476D1CE4E5B9)
        z ^= z >> np.uint64(27)
        z *= np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    b = z.view(np.uint8)
    s = byte_off - 8 * w0
    return b[s:s + n].copy()


def digest(vals: np.ndarray, k_index: np.ndarray | None = None) -> tuple[int, int]:
    """(XOR, sum c_k*(2k+1) mod 2^32) of per-fragment checksums."""
    v = np.asarray(vals, dtype=np.uint64)
    k = np.arange(v.size, dtype=np.uint64) if k_index is None else np.asarray(k_index, dtype=np.uint64)
    x = int(np.bitwise_xor.reduce(v.astype(np.uint32))) if v.size else 0
    s = int(((v * (2 * k + 1)) & np.uint64(0xFFFFFFFF)).sum() & 0xFFFFFFFF) if v.size else 0
    return x, s
