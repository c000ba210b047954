"""lampi_amd -- MI355X-native engine for LA-MPI's per-fragment data-integrity checksums.

Hot path (BASELINE.json north_star): the 32-bit CRC (``uicrc``, CRC-32/MPEG-2) and additive
(``uicsum``) checksums that LA-MPI computes over every message fragment
(ref src/util/MemFunctions.cc, applied in src/path/{gm,ib,quadrics}), as hand-written HIP
kernels for gfx950 behind the C ABI in include/lampi_csum.h (liblampi_csum.so).

* :mod:`lampi_amd.memfunctions` -- the reference's host API (``uicrc``, ``bcopy_uicrc``,
  ``uicsum``, ``bcopy_uicsum``, ``header_checksum``), computed on the GPU.
* :mod:`lampi_amd.device` -- batched device-resident checksums over torch tensors
  (imported lazily: it needs torch).
"""
from ._lib import CRC32, CRC_INITIAL_REGISTER, CRC_POLYNOMIAL, NONE, SUM32, FragDesc, lib  # noqa: F401
from .memfunctions import (PartialState, PartialState64, bcopy_csum, bcopy_uicrc, bcopy_uicsum,  # noqa: F401
                           csum, header_checksum, uicrc, uicsum)

__version__ = "0.1.0"
