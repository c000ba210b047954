"""CPU: the lane algebra the row kernels compute, checked against the oracle's uicrc (no GPU, no library).

crc_regular_kernel cuts a 4 KiB row into 64 lane pieces of 64 bytes.  Lane l keeps a register of its
own: the fragment's register enters as data at lane 0 of its first row, every row the lane's register is shifted by
4,032 zero bytes (the Horner step) and run through the lane's next piece, and at the fragment's end lane l's register
is shifted by 64 (63 - l) zero bytes (its combine column) and the 64 registers are XORed.  The packed rows (4.1.1)
put 64 / kSub fragments of kSub pieces in one row: the register enters at each group's first lane and lane l shifts
by 64 (kSub - 1 - l % kSub) bytes -- the combine column of lane 64 - kSub + l % kSub -- before its group's XOR.  These
tests restate both with the oracle's register update (crc(c, piece) = uicrc(piece, partial=c); a shift by n zero bytes
= uicrc of n zero bytes from c) and compare with the oracle's uicrc of each whole fragment: the identities the
kernels rest on (crc_tables.h: split / combine, init = data injection), at the sizes the kernels use them.
"""
import numpy as np
import pytest

ROW, PIECE = 4096, 64
ZEROS = bytes(ROW)


def _crc(oracle, c, data):
    return oracle.uicrc(np.frombuffer(bytes(data), dtype=np.uint8), partial=c) if len(data) else c


def _shift(oracle, c, n):
    return _crc(oracle, c, ZEROS[:n]) if n else c


def _row_kernel(oracle, frag, init):
    """Config B's lanes over a fragment of R whole rows."""
    R = len(frag) // ROW
    regs = [init if lane == 0 else 0 for lane in range(64)]
    for r in range(R):
        for lane in range(64):
            if r:
                regs[lane] = _shift(oracle, regs[lane], ROW - PIECE)  # the Horner step
            piece = frag[r * ROW + lane * PIECE:r * ROW + (lane + 1) * PIECE]
            regs[lane] = _crc(oracle, regs[lane], piece)
    v = 0
    for lane in range(64):
        v ^= _shift(oracle, regs[lane], PIECE * (63 - lane))  # the lane's combine column
    return v


@pytest.mark.parametrize("R", [1, 2, 3])
def test_row_lanes_equal_uicrc(oracle, R):
    rng = np.random.default_rng(70 + R)
    frag = rng.integers(0, 256, size=R * ROW, dtype=np.uint8).tobytes()
    for init in (0xFFFFFFFF, 0, int(rng.integers(0, 2**32))):
        assert _row_kernel(oracle, frag, init) == _crc(oracle, init, frag)


@pytest.mark.parametrize("ksub", [1, 2, 4, 8, 16, 32])
def test_packed_row_groups_equal_uicrc(oracle, ksub):
    """One 4 KiB row of 64 / ksub fragments of 64 ksub bytes each (config A's 1 KiB is ksub = 16, 64 B is 1)."""
    rng = np.random.default_rng(90 + ksub)
    row = rng.integers(0, 256, size=ROW, dtype=np.uint8).tobytes()
    init = int(rng.integers(0, 2**32))
    L = PIECE * ksub
    for g in range(64 // ksub):
        v = 0
        for j in range(ksub):  # lane l = g ksub + j, piece j of fragment g
            lane = g * ksub + j
            reg = init if j == 0 else 0  # the register enters at the group's first lane
            reg = _crc(oracle, reg, row[lane * PIECE:(lane + 1) * PIECE])
            col = 64 - ksub + (lane % ksub)  # combine column: a shift by 64 (63 - col) = 64 (ksub - 1 - j) bytes
            v ^= _shift(oracle, reg, PIECE * (63 - col))
        assert v == _crc(oracle, init, row[g * L:(g + 1) * L]), (ksub, g)


def test_register_enters_as_data(oracle):
    """crc(s, B) = crc(0, B ^ bytes_BE(s)) for |B| >= 4 -- the injection at lane 0 (crc_tables.h)."""
    rng = np.random.default_rng(7)
    for n in (4, 5, 63, 64, 4096):
        b = bytearray(rng.integers(0, 256, size=n, dtype=np.uint8).tobytes())
        s = int(rng.integers(0, 2**32))
        inj = bytearray(b)
        for i, x in enumerate(s.to_bytes(4, "big")):
            inj[i] ^= x
        assert _crc(oracle, s, b) == _crc(oracle, 0, inj)
