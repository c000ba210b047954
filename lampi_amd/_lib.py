"""ctypes binding of liblampi_csum.so (the C ABI declared in include/lampi_csum.h).

The shared library holds the gfx950 kernels; there is no Python or CPU fallback.  If the
library is missing or cannot be loaded, :func:`lib` raises ``RuntimeError`` -- callers are
expected to fail loudly, never to compute checksums some other way.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LAMPI_CSUM_LIB", os.path.join(_HERE, "liblampi_csum.so"))
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "lampi_csum.h")

CRC32 = 0  # enum lampi_csum_mode (include/lampi_csum.h)
SUM32 = 1
NONE = 2  # checksumming off (doChecksum == false): the copying batches only (send and receive)
BY_BYTES = 0x100  # LAMPI_CSUM_BY_BYTES: byte-balanced descriptor batches (OR'ed into the mode)


def rows_hint_bits(rows: int) -> int:
    """LAMPI_CSUM_ROWS_HINT(rows): OR'ed into the mode of the CRC copy batches (0: no hint)."""
    if not 0 <= int(rows) <= 0xFFF:
        raise ValueError("rows_hint is 0..4095")
    return (int(rows) & 0xFFF) << 16
CRC_POLYNOMIAL = 0x04C11DB7  # ref src/util/MemFunctions.h:36
CRC_INITIAL_REGISTER = 0xFFFFFFFF  # ref src/util/MemFunctions.h:37


class FragDesc(ctypes.Structure):
    """struct lampi_frag_desc (16 bytes): addr u64, length u32, partial u32."""

    _fields_ = [("addr", ctypes.c_uint64), ("length", ctypes.c_uint32), ("partial", ctypes.c_uint32)]


assert ctypes.sizeof(FragDesc) == 16


class CopyDesc(ctypes.Structure):
    """struct lampi_copy_desc (32 bytes): src u64, dst u64, copylen, csumlen, partial, reserved u32."""

    _fields_ = [("src", ctypes.c_uint64), ("dst", ctypes.c_uint64), ("copylen", ctypes.c_uint32),
                ("csumlen", ctypes.c_uint32), ("partial", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


assert ctypes.sizeof(CopyDesc) == 32


class RecvDesc(ctypes.Structure):
    """struct lampi_recv_desc (32 bytes): frag u64, app u64, app_len i64, length u32, reserved u32."""

    _fields_ = [("frag", ctypes.c_uint64), ("app", ctypes.c_uint64), ("app_len", ctypes.c_int64),
                ("length", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


assert ctypes.sizeof(RecvDesc) == 32

class HostRecvFrag(ctypes.Structure):
    """struct lampi_host_recv_frag (32 bytes): frag_off u64, app ptr, app_len i64, length u32, expected u32."""

    _fields_ = [("frag_off", ctypes.c_uint64), ("app", ctypes.c_void_p), ("app_len", ctypes.c_int64),
                ("length", ctypes.c_uint32), ("expected", ctypes.c_uint32)]


assert ctypes.sizeof(HostRecvFrag) == 32


class HostPiece(ctypes.Structure):
    """struct lampi_host_piece (32 bytes): src ptr, dst ptr, copylen, csumlen, partial, reserved u32."""

    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("copylen", ctypes.c_uint32),
                ("csumlen", ctypes.c_uint32), ("partial", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


assert ctypes.sizeof(HostPiece) == 32

_lock = threading.Lock()
_lib = None

c_ulong = ctypes.c_ulong
c_uint = ctypes.c_uint
c_void_p = ctypes.c_void_p
c_size_t = ctypes.c_size_t
PUINT = ctypes.POINTER(ctypes.c_uint)
PULONG = ctypes.POINTER(ctypes.c_ulong)

# name -> (restype, argtypes); the full exported C ABI.
PROTOTYPES = {
    "lampi_uicrc": (c_uint, [c_void_p, c_ulong, c_uint]),
    "lampi_bcopy_uicrc": (c_uint, [c_void_p, c_void_p, c_ulong, c_ulong, c_uint]),
    "lampi_uicsum": (c_uint, [c_void_p, c_ulong, PUINT, PUINT]),
    "lampi_bcopy_uicsum": (c_uint, [c_void_p, c_void_p, c_ulong, c_ulong, PUINT, PUINT]),
    "lampi_csum": (c_ulong, [c_void_p, c_ulong, PULONG, PULONG]),
    "lampi_bcopy_csum": (c_ulong, [c_void_p, c_void_p, c_ulong, c_ulong, PULONG, PULONG]),
    "lampi_frag_csum64_batch": (ctypes.c_int, [c_void_p, c_size_t, c_void_p, c_void_p]),
    "lampi_frag_csum_batch": (ctypes.c_int, [c_void_p, c_size_t, c_void_p, ctypes.c_int, c_void_p]),
    "lampi_frag_bcopy_batch": (ctypes.c_int, [c_void_p, c_size_t, c_void_p, ctypes.c_int, c_void_p]),
    "lampi_msg_bcopy": (ctypes.c_int, [c_void_p, c_size_t, c_size_t, c_void_p, c_size_t, ctypes.c_uint32, c_void_p,
                                       ctypes.c_int, c_void_p]),
    "lampi_chain_csum_batch": (ctypes.c_int, [c_void_p, c_size_t, c_void_p, c_size_t, c_void_p, ctypes.c_int,
                                              c_void_p]),
    "lampi_header_csum_batch": (ctypes.c_int, [c_void_p, c_size_t, c_size_t, ctypes.c_uint32, ctypes.c_uint32, c_void_p,
                                               ctypes.c_int, c_void_p]),
    "lampi_header_check_batch": (ctypes.c_int, [c_void_p, c_size_t, c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                                ctypes.c_uint32, c_void_p, c_void_p, ctypes.c_int, c_void_p]),
    "lampi_header_compare_batch": (ctypes.c_int, [c_void_p, c_size_t, c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                                  c_void_p, c_void_p, ctypes.c_int, c_void_p]),
    "lampi_frag_csum_batch_strided": (ctypes.c_int, [c_void_p, c_size_t, c_void_p, c_size_t, ctypes.c_int, c_void_p]),
    "lampi_frag_bcopy_batch_strided": (ctypes.c_int, [c_void_p, c_size_t, c_void_p, c_size_t, ctypes.c_int, c_void_p]),
    "lampi_msg_bcopy_strided": (ctypes.c_int, [c_void_p, c_size_t, c_size_t, c_void_p, c_size_t, ctypes.c_uint32,
                                               c_void_p, c_size_t, ctypes.c_int, c_void_p]),
    "lampi_chain_csum_batch_strided": (ctypes.c_int, [c_void_p, c_size_t, c_void_p, c_size_t, c_void_p, c_size_t,
                                                      ctypes.c_int, c_void_p]),
    "lampi_header_csum_batch_strided": (ctypes.c_int, [c_void_p, c_size_t, c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                                       c_void_p, c_size_t, ctypes.c_int, c_void_p]),
    "lampi_check_data_batch": (ctypes.c_int, [c_void_p, c_void_p, c_size_t, c_void_p, c_size_t, c_size_t, c_void_p,
                                              c_void_p, c_void_p]),
    "lampi_copy_to_app_batch": (ctypes.c_int, [c_void_p, c_size_t, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p,
                                               c_void_p, ctypes.c_int, c_void_p]),
    "lampi_chain_copy_to_app_batch": (ctypes.c_int, [c_void_p, c_size_t, c_void_p, c_size_t, c_void_p, c_size_t,
                                                     c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_int, c_void_p]),
    "lampi_msg_csum": (ctypes.c_int, [c_void_p, c_size_t, c_size_t, ctypes.c_uint32, c_void_p, ctypes.c_int,
                                      c_void_p]),
    "lampi_fill_stream": (ctypes.c_int, [c_void_p, c_size_t, ctypes.c_uint64, ctypes.c_uint64, c_void_p]),
    "lampi_fill_stream_frags": (ctypes.c_int, [c_void_p, c_size_t, c_size_t, ctypes.c_uint64, ctypes.c_uint64,
                                               ctypes.c_uint64, c_void_p]),
    "lampi_host_release": (None, []),
    "lampi_host_pinned_bytes": (ctypes.c_int64, []),
    "lampi_host_msg_csum": (ctypes.c_int, [c_void_p, c_size_t, c_size_t, c_size_t, c_size_t, ctypes.c_uint32,
                                           c_void_p, ctypes.c_int]),
    "lampi_host_msg_bcopy": (ctypes.c_int, [c_void_p, c_size_t, c_size_t, c_size_t, c_size_t, c_void_p, c_size_t,
                                            ctypes.c_uint32, c_void_p, ctypes.c_int]),
    "lampi_host_copy_to_app_batch": (ctypes.c_int, [c_void_p, c_size_t, c_void_p, c_size_t, c_void_p, c_void_p,
                                                    c_void_p, c_void_p, ctypes.c_int]),
    "lampi_host_header_check_batch": (ctypes.c_int, [c_void_p, c_size_t, c_void_p, c_size_t, ctypes.c_uint32,
                                                     ctypes.c_uint32, ctypes.c_uint32, c_void_p, c_void_p,
                                                     ctypes.c_int]),
    "lampi_host_header_compare_batch": (ctypes.c_int, [c_void_p, c_size_t, c_void_p, c_size_t, ctypes.c_uint32,
                                                       ctypes.c_uint32, c_void_p, c_void_p, ctypes.c_int]),
    "lampi_host_chain_csum_batch": (ctypes.c_int, [c_void_p, c_size_t, c_void_p, c_size_t, c_void_p, ctypes.c_int]),
    "lampi_host_chain_copy_to_app_batch": (ctypes.c_int, [c_void_p, c_size_t, c_void_p, c_size_t, c_void_p, c_void_p,
                                                          c_void_p, c_void_p, c_void_p, ctypes.c_int]),
    "lampi_device_scratch_bytes": (ctypes.c_int64, []),
    "lampi_host_register": (ctypes.c_int, [c_void_p, c_size_t]),
    "lampi_host_unregister": (ctypes.c_int, [c_void_p]),
    "lampi_csum_version": (ctypes.c_char_p, []),
}


def lib() -> ctypes.CDLL:
    """Load (once) and return liblampi_csum.so with prototypes set; raise if absent."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"liblampi_csum.so not found at {LIB_PATH}: build it with "
                    "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
            handle = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in PROTOTYPES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
        return _lib


def check(rc: int, what: str) -> None:
    """Raise on a nonzero hipError_t code returned by a device entry point."""
    if rc != 0:
        raise RuntimeError(f"{what} failed with hipError_t {rc}")
