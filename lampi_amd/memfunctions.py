"""Host-side mirror of LA-MPI's checksum interface (ref src/util/MemFunctions.h:43-65).

Same names, same argument meaning, same return values as the reference overloads, so code
and tests written against the reference read the same here:

=========================  ==================================================  =====================
this module                reference                                           C ABI entry point
=========================  ==================================================  =====================
``uicrc``                  ``uicrc`` MemFunctions.cc:1331-1374                 ``lampi_uicrc``
``bcopy_uicrc``            ``bcopy_uicrc`` MemFunctions.cc:1263-1329           ``lampi_bcopy_uicrc``
``uicsum``                 ``uicsum`` MemFunctions.cc:1073-1231                ``lampi_uicsum``
``bcopy_uicsum``           ``bcopy_uicsum`` MemFunctions.cc:518-893            ``lampi_bcopy_uicsum``
``csum``                   ``csum`` MemFunctions.cc:913-1071 (64-bit words)    ``lampi_csum``
``bcopy_csum``             ``bcopy_csum`` MemFunctions.cc:142-516              ``lampi_bcopy_csum``
``header_checksum``        ``BasePath_t::headerChecksum`` path/common/path.h:280-314
=========================  ==================================================  =====================

Every checksum is computed by the gfx950 kernels in liblampi_csum.so (the bytes are staged
to the GPU and back).  Like the reference, these functions return the checksum and report
no errors; a missing library or GPU raises (library) or aborts (HIP runtime).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from ._lib import CRC_INITIAL_REGISTER, lib

__all__ = [
    "CRC_INITIAL_REGISTER", "PartialState", "PartialState64", "uicrc", "bcopy_uicrc", "uicsum", "bcopy_uicsum",
    "csum", "bcopy_csum", "header_checksum",
]


@dataclass
class PartialState:
    """(lastPartialInt, lastPartialLength) of the reference's additive checksum chaining.

    ``plen`` bytes (1..3) of the current 32-bit word have been summed and ``pint`` is that
    word; the reference keeps these in caller stack variables (src/path/gm/sendFrag.cc:178).
    """

    pint: int = 0
    plen: int = 0


@dataclass
class PartialState64:
    """(lastPartialLong, lastPartialLength) of the 64-bit ``csum`` chaining (plen in 0..7)."""

    plong: int = 0
    plen: int = 0


def _ro_ptr(buf) -> tuple[int, np.ndarray]:
    arr = np.frombuffer(buf, dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf.view(np.uint8).reshape(-1)
    if not arr.flags["C_CONTIGUOUS"]:
        raise ValueError("buffer must be contiguous")
    return arr.ctypes.data, arr


def _rw_ptr(buf) -> tuple[int, np.ndarray]:
    if isinstance(buf, np.ndarray):
        arr = buf.view(np.uint8).reshape(-1)
    else:
        arr = np.frombuffer(buf, dtype=np.uint8)
    if not arr.flags["WRITEABLE"] or not arr.flags["C_CONTIGUOUS"]:
        raise ValueError("destination must be a writable contiguous buffer")
    return arr.ctypes.data, arr


def _check_len(arr: np.ndarray, n: int, what: str) -> None:
    if n < 0 or n > arr.size:
        raise ValueError(f"{what}={n} exceeds the buffer ({arr.size} bytes)")


def uicrc(source, crclen: int | None = None, partial_crc: int = CRC_INITIAL_REGISTER) -> int:
    """CRC-32/MPEG-2 register after ``crclen`` bytes of ``source`` starting from ``partial_crc``."""
    p, arr = _ro_ptr(source)
    n = arr.size if crclen is None else int(crclen)
    _check_len(arr, n, "crclen")
    return int(lib().lampi_uicrc(p, n, partial_crc & 0xFFFFFFFF))


def bcopy_uicrc(source, destination, copylen: int, crclen: int,
                partial_crc: int = CRC_INITIAL_REGISTER) -> int:
    """Copy ``copylen`` bytes and return the CRC of ``max(copylen, crclen)`` bytes of ``source``."""
    ps, a = _ro_ptr(source)
    pd, b = _rw_ptr(destination)
    _check_len(a, max(copylen, crclen), "crclen")
    _check_len(b, copylen, "copylen")
    return int(lib().lampi_bcopy_uicrc(ps, pd, copylen, crclen, partial_crc & 0xFFFFFFFF))


def _state_args(state: PartialState | None):
    st = state if state is not None else PartialState()
    pi = ctypes.c_uint(st.pint & 0xFFFFFFFF)
    pl = ctypes.c_uint(st.plen & 0xFFFFFFFF)
    return st, pi, pl


def uicsum(source, csumlen: int | None = None, state: PartialState | None = None) -> int:
    """32-bit additive checksum increment of ``csumlen`` bytes; ``state`` chains calls (``+=``)."""
    p, arr = _ro_ptr(source)
    n = arr.size if csumlen is None else int(csumlen)
    _check_len(arr, n, "csumlen")
    st, pi, pl = _state_args(state)
    r = int(lib().lampi_uicsum(p, n, ctypes.byref(pi), ctypes.byref(pl)))
    st.pint, st.plen = pi.value, pl.value
    return r


def bcopy_uicsum(source, destination, copylen: int, csumlen: int, state: PartialState | None = None) -> int:
    """Copy ``copylen`` bytes; additive checksum of ``max(copylen, csumlen)`` bytes of ``source``."""
    ps, a = _ro_ptr(source)
    pd, b = _rw_ptr(destination)
    _check_len(a, max(copylen, csumlen), "csumlen")
    _check_len(b, copylen, "copylen")
    st, pi, pl = _state_args(state)
    r = int(lib().lampi_bcopy_uicsum(ps, pd, copylen, csumlen, ctypes.byref(pi), ctypes.byref(pl)))
    st.pint, st.plen = pi.value, pl.value
    return r


def _state64_args(state: PartialState64 | None):
    st = state if state is not None else PartialState64()
    return st, ctypes.c_ulong(st.plong & (2**64 - 1)), ctypes.c_ulong(st.plen & (2**64 - 1))


def csum(source, csumlen: int | None = None, state: PartialState64 | None = None) -> int:
    """64-bit additive checksum increment of ``csumlen`` bytes; ``state`` chains calls (``+=`` mod 2^64)."""
    p, arr = _ro_ptr(source)
    n = arr.size if csumlen is None else int(csumlen)
    _check_len(arr, n, "csumlen")
    st, pl, pn = _state64_args(state)
    r = int(lib().lampi_csum(p, n, ctypes.byref(pl), ctypes.byref(pn)))
    st.plong, st.plen = pl.value, pn.value
    return r


def bcopy_csum(source, destination, copylen: int, csumlen: int, state: PartialState64 | None = None) -> int:
    """Copy ``copylen`` bytes; 64-bit additive checksum of ``max(copylen, csumlen)`` bytes."""
    ps, a = _ro_ptr(source)
    pd, b = _rw_ptr(destination)
    _check_len(a, max(copylen, csumlen), "csumlen")
    _check_len(b, copylen, "copylen")
    st, pl, pn = _state64_args(state)
    r = int(lib().lampi_bcopy_csum(ps, pd, copylen, csumlen, ctypes.byref(pl), ctypes.byref(pn)))
    st.plong, st.plen = pl.value, pn.value
    return r


def header_checksum(header, crclen: int, word_count: int, usecrc: bool) -> int:
    """``BasePath_t::headerChecksum`` (ref src/path/common/path.h:280-314).

    CRC mode: ``uicrc(header, crclen)`` stored byte-swapped, so that the CRC of the header
    followed by the stored value is 0 (receivers test that, src/path/gm/path.cc:379-384).
    Additive mode: the sum of ``word_count`` little-endian 32-bit words.
    """
    if usecrc:
        c = uicrc(header, crclen)
        return int.from_bytes(c.to_bytes(4, "little"), "big")
    return uicsum(header, 4 * word_count)
