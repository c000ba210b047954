"""GPU parity: the gfx950 kernels (through the C ABI) vs the oracle, bit-exact.

Sizes the oracle finishes in seconds are compared fragment by fragment; the BASELINE
config B (4M x 4 KiB, 16 GiB device-resident) is compared through its committed digests
(computed by the reference-pinned oracle).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EDGE_LENS = [0, 1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 63, 64, 65, 127, 1023, 1024, 1025, 1976, 2047, 2048, 4092,
             4095, 4096, 4097, 8191, 8192, 12288, 16383, 16384, 16385, 65455, 65456, 65536]


def _dv():
    from lampi_amd import device as dv

    return dv


def test_stream_generator_matches_oracle(cuda, oracle):
    import torch

    dv = _dv()
    for seed, off, n in [(2, 0, 1 << 16), (7, 13, 99999), (1, 5, 17)]:
        t = torch.empty(n, dtype=torch.uint8, device=cuda)
        dv.fill_stream(t, seed, byte_off=off)
        assert np.array_equal(t.cpu().numpy(), oracle.stream(seed, off, n))
    t = torch.empty(6 * 4096, dtype=torch.uint8, device=cuda)
    dv.fill_stream_frags(t, 6, 4096, seed=3, k0=5, kstep=8)
    want = np.concatenate([oracle.stream(3, (5 + 8 * i) * 4096, 4096) for i in range(6)])
    assert np.array_equal(t.cpu().numpy(), want)


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
@pytest.mark.parametrize("L", [64, 1024, 1976, 4096, 16384, 65456])
def test_uniform_batches(cuda, oracle, mode, L):
    import torch

    dv = _dv()
    n = max(8, (8 << 20) // L)
    buf = torch.empty(n * L, dtype=torch.uint8, device=cuda)
    dv.fill_stream(buf, seed=2)
    got = dv.as_u32(dv.msg_csum(buf, L, mode=mode))
    want = oracle.uniform_batch(2, 0, n, L, mode)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
@pytest.mark.parametrize("L", [4096, 8192, 12288, 16384, 32768, 65536])
def test_regular_batches_every_schedule(cuda, oracle, L, mode):
    """The regular read kernel's schedules (CRC and SUM): 4 KiB batches in 8 KiB row order plus
    the n % 2 tail launch, fragment-order batches for the other multiples of 4 KiB, small-batch
    fpw halving; a random starting register each (CRC)."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(L)
    counts = [1, 2, 3, 4, 5, 7, 9, 97, 1023, 6 * 4 * 4 * 3 + 1] if L == 4096 else [1, 2, 3, 5, 17, 101]
    for n in counts:
        part = int(rng.integers(0, 2**32))
        buf = torch.empty(n * L, dtype=torch.uint8, device=cuda)
        dv.fill_stream(buf, seed=L + n)
        got = dv.as_u32(dv.msg_csum(buf, L, partial=part, mode=mode))
        host = buf.cpu().numpy()
        offs = np.arange(n, dtype=np.uint64) * L
        lens = np.full(n, L, np.uint32)
        want = oracle.desc_batch(host, offs, lens, np.full(n, part, np.uint32) if mode == 0 else None, mode)
        assert np.array_equal(got, want), (L, n, mode)


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
@pytest.mark.parametrize("L", [64, 128, 256, 512, 1024, 2048])
def test_packed_row_messages(cuda, oracle, L, mode):
    """Messages of 64 B .. 2 KiB fragments on config B's kernel in packed rows (round 6: 64 / kSub fragments per
    4 KiB row, crc_regular_kernel<kSub>; SUM up to 1 KiB on sum_row4k_kernel, one short-lived workgroup per 4 KiB):
    whole 8 KiB items (4 KiB rows) through that launch, the rest -- a tail of up to two rows' fragments and a short
    last fragment -- through the other schedules; random registers (CRC), unaligned bases, sizes just at and above
    the minimum (256 rows)."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(L + 7 * mode)
    cases = [(256 * 4096, 0), (256 * 4096 + 3 * L + 17, 0), (257 * 4096 + L, 0), (600 * 4096 + 1, 0),
             (300 * 4096 + 5 * L, 4), (300 * 4096, 3), (255 * 4096 + 4 * L + 1, 0)]
    for msg_len, off in cases:
        part = int(rng.integers(0, 2**32))
        buf = torch.empty(msg_len + off, dtype=torch.uint8, device=cuda)
        dv.fill_stream(buf, seed=msg_len + L)
        got = dv.as_u32(dv.msg_csum(buf[off:], L, partial=part, mode=mode))
        host = buf.cpu().numpy()
        n = (msg_len + L - 1) // L
        offs = off + np.arange(n, dtype=np.uint64) * L
        lens = np.minimum(L, msg_len + off - offs).astype(np.uint32)
        want = oracle.desc_batch(host, offs, lens, np.full(n, part, np.uint32) if mode == 0 else None, mode)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (L, msg_len, off, bad[:8].tolist())


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_config_a_shape_full_digest(cuda, mode):
    """Config A's workload on the GPU (1M x 1 KiB, stream seed 1: BASELINE.md's digest feb61101 / 41fadf13 in CRC,
    tests/golden/bench_digests.json in SUM) through the message entry point (packed rows)."""
    import json

    import torch

    from oracle.oracle import digest

    dv = _dv()
    n, L = 1048576, 1024
    buf = torch.empty(n * L, dtype=torch.uint8, device=cuda)
    dv.fill_stream(buf, seed=1)
    v = dv.as_u32(dv.msg_csum(buf, L, mode=mode))
    if mode == 0:
        assert digest(v) == (0xFEB61101, 0x41FADF13)
    else:
        with open(os.path.join(os.path.dirname(__file__), "golden", "bench_digests.json")) as f:
            e = [x for x in json.load(f)["entries"] if (x["seed"], x["n_total"], x["frag_bytes"], x["mode"]) ==
                 (1, n, L, "sum") and "nshard" not in x][0]
        assert digest(v) == (e["xor"], e["wsum"])


@pytest.mark.parametrize("L", [1, 3, 15, 16, 17, 63, 64, 1976, 4095, 4096, 4097, 16384, 65456, (1 << 20) + 48])
def test_sum_messages_short_lived_workgroups(cuda, oracle, L):
    """lampi_msg_csum SUM of messages of >= 256 fragments (one fragment per short-lived 128-thread workgroup,
    round 5): lengths around the 16-byte chunk, the 4 KiB row and large fragments, a ragged last fragment, a
    message start at every offset 0..15 of a 16-byte line; every fragment vs the oracle."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(L)
    nf = 256 + int(rng.integers(0, 40))
    for shift in (0, 1, 7, 13):
        msg_len = (nf - 1) * L + int(rng.integers(1, L + 1))
        raw = torch.empty(msg_len + 16, dtype=torch.uint8, device=cuda)
        dv.fill_stream(raw, seed=L + shift)
        buf = raw[shift:shift + msg_len]
        got = dv.as_u32(dv.msg_csum(buf, L, mode=dv.SUM32))
        host = buf.cpu().numpy()
        offs = np.arange(nf, dtype=np.uint64) * L
        lens = np.minimum(L, msg_len - offs.astype(np.int64)).astype(np.uint32)
        want = oracle.desc_batch(host, offs, lens, None, 1)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (L, shift, bad[:8].tolist())


@pytest.mark.parametrize("L,nf", [(4097, 4100), (16384, 4096), (32767, 4111), (36864, 4096), (16384, 300),
                                  (65456, 700), ((1 << 20) + 48, 300), (3 << 20, 40)])
def test_sum_multirow_schedules(cuda, oracle, L, nf):
    """Read-only SUM of fragments over one 4 KiB row (sum_ro_groups, round 5): 2-8 rows in batches of
    >= 4,096 one per short-lived workgroup; otherwise row groups widened until the launch has 65,536
    workgroups (groups of >= 2 rows).  Messages (ragged last fragment, odd start) and descriptors at random
    byte offsets with the caller's rows hint; every fragment vs the oracle."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(L + nf)
    msg_len = (nf - 1) * L + int(rng.integers(1, L + 1))
    raw = torch.empty(msg_len + 16, dtype=torch.uint8, device=cuda)
    dv.fill_stream(raw, seed=L ^ nf)
    buf = raw[5:5 + msg_len]
    host = buf.cpu().numpy()
    offs = np.arange(nf, dtype=np.uint64) * L
    lens = np.minimum(L, msg_len - offs.astype(np.int64)).astype(np.uint64)
    want = oracle.desc_batch(host, offs, lens.astype(np.uint32), None, 1)
    got = dv.as_u32(dv.msg_csum(buf, L, mode=dv.SUM32))
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, ("msg", L, nf, bad[:8].tolist())
    # descriptors: the same fragments shuffled, lengths trimmed by up to 15 bytes, the caller's hint
    perm = rng.permutation(nf)
    offs2, lens2 = offs[perm], lens[perm]
    lens2 = lens2 - np.minimum(lens2, rng.integers(0, 16, size=nf).astype(np.uint64))
    descs = dv.make_descs(buf, offs2, lens2, np.zeros(nf, np.uint64))
    want2 = oracle.desc_batch(host, offs2, lens2.astype(np.uint32), None, 1)
    rows = (L + 4095) // 4096
    got2 = dv.as_u32(dv.frag_csum_batch(descs, mode=dv.SUM32, rows_hint=rows))
    bad = np.nonzero(got2 != want2)[0]
    assert bad.size == 0, ("desc", L, nf, bad[:8].tolist())


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_message_with_short_last_fragment(cuda, oracle, mode):
    import torch

    dv = _dv()
    for msg_len, L in [(1 << 20, 65456), (1000003, 4096), (5, 4096), (4096 * 7 + 1, 4096)]:
        buf = torch.empty(msg_len, dtype=torch.uint8, device=cuda)
        dv.fill_stream(buf, seed=11)
        got = dv.as_u32(dv.msg_csum(buf, L, partial=0x12345678, mode=mode))
        host = buf.cpu().numpy()
        nf = (msg_len + L - 1) // L
        offs = np.arange(nf, dtype=np.uint64) * L
        lens = np.minimum(L, msg_len - offs.astype(np.int64)).astype(np.uint32)
        want = oracle.desc_batch(host, offs, lens, np.full(nf, 0x12345678, np.uint32) if mode == 0 else None, mode)
        assert np.array_equal(got, want), (msg_len, L)


@pytest.mark.parametrize("msg_len,L", [
    (65456 * 300, 65456),                  # GM payloads: 16-row frames, 80 bytes of front padding
    (65456 * 300 + 1280, 65456),           # a 1,280-byte last fragment: 15 whole padding rows
    (((1 << 20) + 48) * 5 + 4096 * 3 + 16, (1 << 20) + 48),  # 257-row frames: 17 groups, joined
    ((12288 + 80) * 700 + 16, 12288 + 80),  # 4-row frames, P = 4016: the register in row 0, lane 62
    ((16384 + 1008) * 333, 16384 + 1008),  # P = 3088: lane 48, chunk 1
    ((12288 * 2 + 16) * 97 + 12288 * 2, 12288 * 2 + 16),  # last fragment exactly 6 rows
    ((40000 // 16 * 16) * 777 + 4096, 40000 // 16 * 16),
    ((1 << 20) * 6, 1 << 20),                 # whole-row fragments, 256 rows: 32 groups of 8 rows
    ((1 << 20) * 3 + 4096 * 5 + 7, 1 << 20),  # ... and a last fragment of 5 rows + 7 bytes
    ((131072 - 16) * 40 + 999, 131072 - 16),  # 32 rows, P = 16: 4 groups, the register in group 0
])
def test_message_large_ragged_fragments(cuda, oracle, msg_len, L):
    """lampi_msg_csum CRC of messages of large fragments (GM payloads, 257-row fragments, registers
    landing in every lane and chunk position of a 4 KiB frame, last fragments of a few rows or exactly
    whole rows; from 8 rows the read-only table-light kernel, above 16 rows as 8-row groups joined),
    every fragment vs the oracle, two registers."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(msg_len)
    buf = torch.empty(msg_len, dtype=torch.uint8, device=cuda)
    dv.fill_stream(buf, seed=msg_len % 1000)
    host = buf.cpu().numpy()
    nf = (msg_len + L - 1) // L
    offs = np.arange(nf, dtype=np.uint64) * L
    lens = np.minimum(L, msg_len - offs.astype(np.int64)).astype(np.uint32)
    for part in (0xFFFFFFFF, int(rng.integers(0, 2**32))):
        got = dv.as_u32(dv.msg_csum(buf, L, partial=part))
        want = oracle.desc_batch(host, offs, lens, np.full(nf, part, np.uint32), 0)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (msg_len, L, hex(part), bad[:8].tolist(), nf)


@pytest.mark.parametrize("msg_len,L", [
    (65456 * 4102 + 1280, 65456),           # GM payloads, >= 256 MiB (the table-light kernel); the
                                            # short last fragment's register lands in row 15
    (39984 * 6800 + 4096 * 3 + 16, 39984),  # 10-row frames, P = 976; last fragment 3 rows + 16 bytes
    ((131072 - 16) * 2100, 131072 - 16),    # 32-row frames, P = 16 (8-row groups)
    (24592 * 11000 + 4096 + 32, 24592),     # 7-row frames (P = 4080): the framed regular kernel
    (20480 * 13200 + 48, 20480 - 16),       # 5-row frames, P = 16, ragged end: the same
])
def test_message_frames_regular_kernel(cuda, oracle, msg_len, L):
    """lampi_msg_csum CRC of >= 256 MiB messages of 20-128 KiB fragments that are not whole rows
    (under 8 rows crc_regular_kernel<kFrame>: 4 KiB frames read through buffer descriptors, the
    register injected at the frame padding's end; from 8 rows the table-light kernel), every fragment
    vs the oracle, two registers."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(L)
    buf = torch.empty(msg_len, dtype=torch.uint8, device=cuda)
    dv.fill_stream(buf, seed=L % 977)
    host = buf.cpu().numpy()
    nf = (msg_len + L - 1) // L
    offs = np.arange(nf, dtype=np.uint64) * L
    lens = np.minimum(L, msg_len - offs.astype(np.int64)).astype(np.uint32)
    for part in (0xFFFFFFFF, int(rng.integers(0, 2**32))):
        got = dv.as_u32(dv.msg_csum(buf, L, partial=part))
        want = oracle.desc_batch(host, offs, lens, np.full(nf, part, np.uint32), 0)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (msg_len, L, hex(part), bad[:8].tolist(), nf)


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_descriptor_batch_edges_and_alignment(cuda, oracle, mode):
    import torch

    dv = _dv()
    rng = np.random.default_rng(1234)
    base = torch.empty(4 << 20, dtype=torch.uint8, device=cuda)
    dv.fill_stream(base, seed=21)
    host = base.cpu().numpy()
    lens, offs = [], []
    for L in EDGE_LENS:
        for a in range(0, 17):  # every alignment mod 16 plus one
            lens.append(L)
            offs.append(int(rng.integers(0, (4 << 20) - 70000)) // 64 * 64 + a)
    lens = np.array(lens, dtype=np.uint64)
    offs = np.array(offs, dtype=np.uint64)
    parts = rng.integers(0, 2**32, size=lens.size, dtype=np.uint64)
    parts[::3] = 0xFFFFFFFF
    descs = dv.make_descs(base, offs, lens, parts)
    want = oracle.desc_batch(host, offs, lens, parts.astype(np.uint32) if mode == 0 else None, mode)
    by_bytes = lambda d, mode: dv.frag_csum_batch(d, mode=mode, by_bytes=True)  # noqa: E731
    # piece streams (count split, byte plan) / one wave per fragment
    for name, fn in (("count", dv.frag_csum_batch), ("bytes", by_bytes), ("per_wave", dv.diag_frag_csum_batch_per_wave)):
        got = dv.as_u32(fn(descs, mode=mode))
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (name, [(int(lens[i]), int(offs[i]) % 16) for i in bad[:10]])


def test_descriptor_batch_random(cuda, oracle):
    import torch

    dv = _dv()
    rng = np.random.default_rng(99)
    base = torch.empty(64 << 20, dtype=torch.uint8, device=cuda)
    dv.fill_stream(base, seed=33)
    host = base.cpu().numpy()
    n = 20000
    lens = rng.integers(0, 70000, size=n).astype(np.uint64)
    offs = rng.integers(0, (64 << 20) - 70000, size=n).astype(np.uint64)
    parts = rng.integers(0, 2**32, size=n, dtype=np.uint64)
    descs = dv.make_descs(base, offs, lens, parts)
    for mode in (0, 1):
        want = oracle.desc_batch(host, offs, lens, parts.astype(np.uint32) if mode == 0 else None, mode)
        for by_bytes in (False, True):
            got = dv.as_u32(dv.frag_csum_batch(descs, mode=mode, by_bytes=by_bytes))
            assert np.array_equal(got, want), by_bytes


@pytest.mark.parametrize("n", [1023, 1024, 5000, 65536, 65537])
def test_descriptor_batch_size_split(cuda, oracle, n):
    """Read-only CRC batches of 1,024..65,536 descriptors run in two launches by size class (DESIGN.md 4.2:
    8-16-row fragments on the table-light kernel, the rest on the piece streams, each skipping the other's):
    the class boundaries 28,672 / 28,673 and 65,536 / 65,537 bytes, empty and tiny fragments, any alignment,
    random registers -- and the batch sizes on either side of the split's range -- against the oracle."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(n)
    base = torch.empty(96 << 20, dtype=torch.uint8, device=cuda)
    dv.fill_stream(base, seed=34)
    host = base.cpu().numpy()
    edge = np.array([0, 1, 15, 16, 4095, 28671, 28672, 28673, 40000, 65455, 65456, 65535, 65536, 65537, 70000],
                    np.uint64)
    lens = np.where(rng.random(n) < 0.5, rng.choice(edge, size=n), rng.integers(0, 70000, size=n)).astype(np.uint64)
    offs = rng.integers(0, (96 << 20) - 70001, size=n).astype(np.uint64)
    parts = rng.integers(0, 2**32, size=n, dtype=np.uint64)
    descs = dv.make_descs(base, offs, lens, parts)
    want = oracle.desc_batch(host, offs, lens, parts.astype(np.uint32), 0)
    got = dv.as_u32(dv.frag_csum_batch(descs, mode=0))
    assert np.array_equal(got, want)


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
@pytest.mark.parametrize("case", ["three", "aligned40", "mixed600", "huge_first"])
def test_descriptor_batch_fragments_across_chains(cuda, oracle, case, mode):
    """The piece-stream kernel cuts a workgroup's pieces into eight chains of equal row counts, so
    a long fragment is checksummed in parts by several chains and joined at the end (stream_join,
    shifts by arbitrary piece counts).  Few fragments per workgroup and multi-MiB lengths make
    fragments span two to eight chains; misaligned ends take the five-load variant."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(hash(case) % 2**32)
    MiB = 1 << 20
    if case == "three":
        lens = np.array([20 * MiB + 3, 1, 5 * MiB + 61], dtype=np.uint64)
        offs = np.array([5, 21 * MiB + 7, 22 * MiB + 1], dtype=np.uint64)
    elif case == "aligned40":
        lens = np.where(np.arange(40) % 2 == 0, 64 * rng.integers(16384, 65536, size=40),
                        64 * rng.integers(1, 20, size=40)).astype(np.uint64)
        offs = (np.concatenate([[0], np.cumsum(lens)[:-1]]) + 4096).astype(np.uint64)
    elif case == "mixed600":
        lens = np.where(rng.integers(0, 8, size=600) == 0, rng.integers(MiB // 2, 3 * MiB, size=600),
                        rng.integers(0, 5000, size=600)).astype(np.uint64)
        offs = rng.integers(0, 40 * MiB, size=600).astype(np.uint64)
    else:  # one fragment much longer than the rest of its workgroup, then empties and tiny ones
        lens = np.array([30 * MiB + 64, 0, 3, 0, 64, 128, 4096, 1], dtype=np.uint64)
        offs = np.array([64, 0, 9, 0, 31 * MiB, 31 * MiB + 64, 31 * MiB + 256, 33 * MiB], dtype=np.uint64)
    size = int((offs + lens).max()) + 64
    base = torch.empty(size, dtype=torch.uint8, device=cuda)
    dv.fill_stream(base, seed=77)
    host = base.cpu().numpy()
    parts = rng.integers(0, 2**32, size=lens.size, dtype=np.uint64)
    descs = dv.make_descs(base, offs, lens, parts)
    want = oracle.desc_batch(host, offs, lens, parts.astype(np.uint32) if mode == 0 else None, mode)
    by_bytes = lambda d, mode: dv.frag_csum_batch(d, mode=mode, by_bytes=True)  # noqa: E731
    # piece streams (count split, byte plan) / one wave per fragment
    for name, fn in (("count", dv.frag_csum_batch), ("bytes", by_bytes), ("per_wave", dv.diag_frag_csum_batch_per_wave)):
        got = dv.as_u32(fn(descs, mode=mode))
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (name, [(int(lens[i]), int(offs[i]) % 16) for i in bad[:10]])


def test_descriptor_batch_maximum_length(cuda):
    """A single fragment of 2^32 - 1 bytes (the largest `length`), with neighbours: its checksum
    must equal the chained checksum of two parts (CRC: the first part's register is the second's
    starting register, crc(s, A||B) = crc(crc(s, A), B); SUM: the sums add when |A| % 4 == 0) --
    a size-independent property at the size where piece indices exceed 2^26 per workgroup and the
    parts of one fragment are joined across all twelve chains (shifts by millions of pieces)."""
    import torch

    dv = _dv()
    L = 2**32 - 1
    base = torch.empty(L + 4096, dtype=torch.uint8, device=cuda)
    dv.fill_stream(base, seed=123)
    a = 1_500_000_004  # first part (a multiple of 4)
    for mode in (dv.CRC32, dv.SUM32):
        whole = dv.make_descs(base, np.array([17, 0, 5], np.uint64), np.array([L, 0, 999], np.uint64),
                              np.array([0xFFFFFFFF, 7, 0x1234], np.uint64))
        w = dv.as_u32(dv.frag_csum_batch(whole, mode=mode))
        first = dv.make_descs(base, np.array([17], np.uint64), np.array([a], np.uint64),
                              np.array([0xFFFFFFFF], np.uint64))
        x = int(dv.as_u32(dv.frag_csum_batch(first, mode=mode))[0])
        second = dv.make_descs(base, np.array([17 + a], np.uint64), np.array([L - a], np.uint64),
                               np.array([x if mode == dv.CRC32 else 0], np.uint64))
        y = int(dv.as_u32(dv.frag_csum_batch(second, mode=mode))[0])
        want = y if mode == dv.CRC32 else (x + y) & 0xFFFFFFFF
        assert int(w[0]) == want, (mode, hex(int(w[0])), hex(want))
        assert int(w[1]) == (7 if mode == dv.CRC32 else 0)  # empty: the register / 0
    del base
    torch.cuda.empty_cache()


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
@pytest.mark.parametrize("case", ["one_huge", "few_huge_ragged", "gm_65456", "mb4_x256", "huge_among_tiny"])
def test_descriptor_batch_byte_balanced(cuda, oracle, case, mode):
    """With LAMPI_CSUM_BY_BYTES, batches of up to 32,768 descriptors are planned by bytes (plan_kernel): fragments longer than
    the plan's window are cut into segments checksummed by different workgroups -- CRC segments from
    the fragment's end, the first from the fragment's register, the others from 0, each part shifted
    past the rest of its fragment and XORed into out[f]; SUM segments from its start, added.  Every
    fragment against the oracle (or, for the 1 GiB batches, against lampi_msg_csum over the same
    bytes, an independent kernel, and a sample against the oracle)."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(abs(hash(case)) % 2**32)
    MiB = 1 << 20
    if case == "one_huge":  # one Quadrics-sized checksum-only send at an odd address
        lens = np.array([9 * MiB + 13], np.uint64)
        offs = np.array([7], np.uint64)
    elif case == "few_huge_ragged":
        lens = np.array([3 * MiB + 1, 0, 17 * MiB + 4095, 2, 6 * MiB, 64 * 1024 + 5, 1 * MiB], np.uint64)
        offs = (np.concatenate([[3], np.cumsum(lens)[:-1] + 3]) + np.arange(lens.size) * 1) .astype(np.uint64)
    elif case == "gm_65456":  # 1 GiB of GM payload-sized fragments (a 1 GiB message, 16,404 fragments)
        n = (1 << 30) // 65456
        lens = np.full(n, 65456, np.uint64)
        offs = np.arange(n, dtype=np.uint64) * np.uint64(65456)
    elif case == "mb4_x256":  # 1 GiB of 4 MiB fragments
        lens = np.full(256, 4 * MiB, np.uint64)
        offs = np.arange(256, dtype=np.uint64) * np.uint64(4 * MiB)
    else:  # a few huge fragments among thousands of tiny ones and empties
        n = 5000
        lens = rng.integers(0, 600, size=n).astype(np.uint64)
        big = rng.choice(n, size=6, replace=False)
        lens[big] = rng.integers(2 * MiB, 12 * MiB, size=6)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64) + np.uint64(1)
    size = int((offs + lens).max()) + 64
    base = torch.empty(size, dtype=torch.uint8, device=cuda)
    dv.fill_stream(base, seed=55)
    parts = rng.integers(0, 2**32, size=lens.size, dtype=np.uint64)
    if case in ("gm_65456", "mb4_x256"):
        parts[:] = 0xFFFFFFFF
    descs = dv.make_descs(base, offs, lens, parts)
    got = dv.as_u32(dv.frag_csum_batch(descs, mode=mode, by_bytes=True))
    if case in ("gm_65456", "mb4_x256"):
        L = int(lens[0])
        want = dv.as_u32(dv.msg_csum(base[:lens.size * L], L, mode=mode))
        assert np.array_equal(got, want)
        idx = rng.choice(lens.size, size=24, replace=False)
        host = base[:lens.size * L].cpu().numpy()
        ref = oracle.desc_batch(host, offs[idx], lens[idx], parts[idx].astype(np.uint32) if mode == 0 else None, mode)
        assert np.array_equal(got[idx], ref)
    else:
        host = base.cpu().numpy()
        want = oracle.desc_batch(host, offs, lens, parts.astype(np.uint32) if mode == 0 else None, mode)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, [(int(lens[i]), int(offs[i]) % 16) for i in bad[:10]]
    # the same batch again on a fresh output (split fragments are accumulated into out: the plan zeroes them)
    out = torch.full((lens.size,), -1, dtype=torch.int32, device=cuda)
    dv.frag_csum_batch(descs, mode=mode, out=out, by_bytes=True)
    assert np.array_equal(dv.as_u32(out), got)
    # and the default count split gives the same values
    assert np.array_equal(dv.as_u32(dv.frag_csum_batch(descs, mode=mode)), got)


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
@pytest.mark.parametrize("case", ["one_64mib", "n16_ragged", "n255_mixed", "n200_tiny", "n3_rows"])
def test_descriptor_small_batch_row_groups(cuda, oracle, case, mode):
    """Read-only descriptor batches under 256 fragments without a rows hint (round 5): every fragment as W
    row groups (W = 4096 for one fragment down to 16 for 255), groups past a fragment's rows empty; CRC on
    the table-light kernel (empty workgroups leave before staging tables) joined by the constant-product
    XOR, SUM groups added.  Odd addresses, ragged and zero lengths, random registers; vs the oracle."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(abs(hash(case)) % 2**32)
    MiB = 1 << 20
    if case == "one_64mib":
        lens = np.array([64 * MiB - 5], np.uint64)
    elif case == "n16_ragged":
        lens = (rng.integers(1, 3 * MiB, size=16) | 1).astype(np.uint64)
        lens[3], lens[7] = 0, 4096 * 4096  # an empty fragment; 4,096 rows: one per group at W = 256
    elif case == "n255_mixed":
        lens = rng.integers(0, 5000, size=255).astype(np.uint64)
        lens[rng.choice(255, size=5, replace=False)] = rng.integers(MiB, 4 * MiB, size=5)
    elif case == "n200_tiny":
        lens = rng.integers(0, 4097, size=200).astype(np.uint64)
    else:  # rows around the group size: 3 fragments at W = 2048
        lens = np.array([2048 * 4096 + 1, 2047 * 4096, 4095 * 4096 + 4095], np.uint64)
    offs = (np.concatenate([[0], np.cumsum(lens)[:-1]]) + np.arange(lens.size) * 3 + 1).astype(np.uint64)
    base = torch.empty(int((offs + lens).max()) + 64, dtype=torch.uint8, device=cuda)
    dv.fill_stream(base, seed=lens.size)
    parts = rng.integers(0, 2**32, size=lens.size, dtype=np.uint64)
    descs = dv.make_descs(base, offs, lens, parts)
    got = dv.as_u32(dv.frag_csum_batch(descs, mode=mode))
    host = base.cpu().numpy()
    want = oracle.desc_batch(host, offs, lens.astype(np.uint32), parts.astype(np.uint32) if mode == 0 else None, mode)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(lens[i]), int(offs[i]) % 16) for i in bad[:10]]
    if case == "one_64mib":  # the schedule itself: ~0.17 ms (CRC) / 0.03 ms (SUM) as row groups, 3.0 / 1.8 ms on
        # the count split (one workgroup for the whole fragment) -- a 1.5 ms bound catches a fall-back
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            dv.frag_csum_batch(descs, mode=mode)
        e1.record()
        torch.cuda.synchronize()
        assert e0.elapsed_time(e1) / 5 < 1.5, e0.elapsed_time(e1) / 5


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
def test_descriptor_batch_row_segments(cuda, oracle, mode):
    """LAMPI_CSUM_ROWS_HINT on lampi_frag_csum_batch: workgroups sized by the hinted length, and above 16
    rows ceil(hint / 16) row segments per fragment computed on the device (CRC cut from the end, SUM from
    the start; split fragments XORed / added into a zeroed out), items past a fragment's last segment
    skipped; CRC from hint 8 on: the read-only table-light kernel, one wave per 8 rows (up to 16 rows:
    one wave per fragment, however long), groups joined by crc_light_group_join_kernel -- the edge
    lengths x alignments with random registers at hints 3, 8, 12, 17, 33 and 49, then random fragments
    of up to ~300 KB at hint 70, every fragment against the oracle."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(4242 + mode)
    base = torch.empty(8 << 20, dtype=torch.uint8, device=cuda)
    dv.fill_stream(base, seed=25)
    host = base.cpu().numpy()
    lens, offs = [], []
    for L in EDGE_LENS + [70001, 131072, 200003]:
        for a in range(0, 17, 4):
            lens.append(L)
            offs.append(int(rng.integers(0, (8 << 20) - 210000)) // 64 * 64 + a)
    lens = np.array(lens, dtype=np.uint64)
    offs = np.array(offs, dtype=np.uint64)
    parts = rng.integers(0, 2**32, size=lens.size, dtype=np.uint64)
    descs = dv.make_descs(base, offs, lens, parts)
    want = oracle.desc_batch(host, offs, lens, parts.astype(np.uint32) if mode == 0 else None, mode)
    for hint in (3, 8, 12, 17, 33, 49):
        got = dv.as_u32(dv.frag_csum_batch(descs, mode=mode, rows_hint=hint))
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (hint, [(int(lens[i]), int(offs[i]) % 16) for i in bad[:10]])
    n = 3000
    lens = rng.integers(0, 300000, size=n).astype(np.uint64)
    offs = rng.integers(0, (8 << 20) - 300001, size=n).astype(np.uint64)
    parts = rng.integers(0, 2**32, size=n, dtype=np.uint64)
    descs = dv.make_descs(base, offs, lens, parts)
    want = oracle.desc_batch(host, offs, lens, parts.astype(np.uint32) if mode == 0 else None, mode)
    out = torch.full((n,), -1, dtype=torch.int32, device=cuda)  # (the launcher zeroes it)
    got = dv.as_u32(dv.frag_csum_batch(descs, mode=mode, out=out, rows_hint=70))
    assert np.array_equal(got, want)


def test_descriptor_batch_row_segments_large(cuda, oracle):
    """The hint at the sizes it is for: 1 GiB of GM's 65,456-byte fragments (hint 16: workgroups of 6
    fragments) and of 4 MiB fragments (hint 1024: 64 segments of 16 rows each; CRC 128 groups of 8)
    and one 2^32 - 1-byte fragment among neighbours (hint 4095: 256 segments of 4,096 rows, CRC 512
    groups of 2,048; shifts past a million rows),
    against lampi_msg_csum / the plain batch over the same bytes and an oracle sample; both modes."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(77)
    buf = torch.empty(1 << 30, dtype=torch.uint8, device=cuda)
    dv.fill_stream(buf, seed=19)
    for L, hint in ((65456, 16), (4 << 20, 1024)):
        n = (1 << 30) // L
        offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
        descs = dv.make_descs(buf, offs, np.full(n, L, np.uint64))
        idx = rng.choice(n, size=min(n, 12), replace=False)
        host = buf[:n * L].cpu().numpy()
        for mode in (dv.CRC32, dv.SUM32):
            got = dv.as_u32(dv.frag_csum_batch(descs, mode=mode, rows_hint=hint))
            assert np.array_equal(got, dv.as_u32(dv.msg_csum(buf[:n * L], L, mode=mode))), (L, mode)
            ref = oracle.desc_batch(host, offs[idx], np.full(idx.size, L, np.uint64),
                                    np.full(idx.size, 0xFFFFFFFF, np.uint32) if mode == dv.CRC32 else None, mode)
            assert np.array_equal(got[idx], ref), (L, mode)
    del buf
    torch.cuda.empty_cache()
    L = 2**32 - 1
    base = torch.empty(L + 4096, dtype=torch.uint8, device=cuda)
    dv.fill_stream(base, seed=123)
    descs = dv.make_descs(base, np.array([17, 0, 5], np.uint64), np.array([L, 0, 999], np.uint64),
                          np.array([0xFFFFFFFF, 7, 0x1234], np.uint64))
    for mode in (dv.CRC32, dv.SUM32):
        want = dv.as_u32(dv.frag_csum_batch(descs, mode=mode))
        got = dv.as_u32(dv.frag_csum_batch(descs, mode=mode, rows_hint=4095))
        assert np.array_equal(got, want), mode
    del base
    torch.cuda.empty_cache()


def test_descriptor_batch_two_buffers(cuda, oracle):
    """Fragments from two buffers more than 2 GiB apart, interleaved in runs so workgroups hold both,
    with lengths at the 64-byte-piece edges that round 3's packed-row experiment (crc_list_kernel,
    DESIGN.md §11) keyed on (64, 1024, 1088, 2048, 2112 bytes), odd lengths beside them,
    empty fragments and random registers.  Every fragment against the oracle."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(64)
    MiB = 1 << 20
    a = torch.empty(8 * MiB, dtype=torch.uint8, device=cuda)
    gap = torch.empty(3 << 30, dtype=torch.uint8, device=cuda)  # pushes b past a's 2 GiB window
    b = torch.empty(8 * MiB, dtype=torch.uint8, device=cuda)
    dv.fill_stream(a, seed=61)
    dv.fill_stream(b, seed=62)
    far = abs(b.data_ptr() - a.data_ptr()) >= (1 << 31)

    def batch(n):
        edges = np.array([64, 128, 960, 1024, 1088, 1984, 2048, 2112, 4096, 0, 1000, 2047, 63, 5000], np.uint64)
        lens = np.where(rng.integers(0, 4, size=n) == 0, rng.choice(edges, size=n),
                        64 * rng.integers(1, 40, size=n)).astype(np.uint64)
        offs = rng.integers(0, 8 * MiB - 6000, size=n).astype(np.uint64)
        offs[rng.integers(0, 3, size=n) > 0] &= ~np.uint64(63)
        parts = rng.integers(0, 2**32, size=n, dtype=np.uint64)
        return lens, offs, parts

    la, oa, pa = batch(24000)
    lb, ob, pb = batch(24000)
    # interleave the two buffers in runs, so some workgroups hold fragments of both
    order = np.argsort(np.concatenate([np.arange(24000) // 5 * 2, np.arange(24000) // 7 * 2 + 1]), kind="stable")
    descs = torch.cat([dv.make_descs(a, oa, la, pa), dv.make_descs(b, ob, lb, pb)])[torch.from_numpy(order).to(cuda)]
    want = np.concatenate([oracle.desc_batch(a.cpu().numpy(), oa, la, pa.astype(np.uint32), 0),
                           oracle.desc_batch(b.cpu().numpy(), ob, lb, pb.astype(np.uint32), 0)])[order]
    for by_bytes in (False, True):
        got = dv.as_u32(dv.frag_csum_batch(descs, mode=dv.CRC32, by_bytes=by_bytes))
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (by_bytes, far, bad[:10])
    del gap
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n", [30000, 300000])
def test_descriptor_batch_small_fragments(cuda, oracle, n):
    """Fragments of 16..1024 bytes (multiples of 16, 16-byte aligned) mixed with unaligned,
    odd-length, empty and multi-row fragments in one batch, every register random: rows hold many
    fragment boundaries (the boundary-mask path and the segmented scan), with misaligned ones in
    the same workgroups.  30,000 runs with 8 fragments per workgroup, 300,000 with the full 256
    (frags_per_wg); both checksum modes."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(2024)
    base = torch.empty(32 << 20, dtype=torch.uint8, device=cuda)
    dv.fill_stream(base, seed=44)
    host = base.cpu().numpy()
    kind = rng.integers(0, 10, size=n)
    lens = np.where(kind < 6, 16 * rng.integers(1, 65, size=n),            # pack members
                    np.where(kind < 8, rng.integers(1, 1100, size=n),       # small, any length
                             rng.integers(0, 20000, size=n))).astype(np.uint64)
    offs = rng.integers(0, (32 << 20) - 20100, size=n).astype(np.uint64)
    offs[kind < 6] &= ~np.uint64(15)                                         # aligned members
    offs[kind == 6] |= np.uint64(1)                                          # misaligned small ones
    parts = rng.integers(0, 2**32, size=n, dtype=np.uint64)
    descs = dv.make_descs(base, offs, lens, parts)
    for mode in (dv.CRC32, dv.SUM32):
        want = oracle.desc_batch(host, offs, lens, parts.astype(np.uint32) if mode == dv.CRC32 else None, mode)
        for by_bytes in (False, True):  # (above 32,768 descriptors the byte plan falls back to the count split)
            got = dv.as_u32(dv.frag_csum_batch(descs, mode=mode, by_bytes=by_bytes))
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, [(mode, by_bytes, int(lens[i]), int(offs[i]) % 16) for i in bad[:10]]


@pytest.mark.parametrize("mode", [0, 1], ids=["crc", "sum"])
@pytest.mark.parametrize("L", [64, 128, 256, 512, 1024, 1976])
def test_small_fragment_sizes_mixed_with_large(cuda, oracle, L, mode):
    """fragments of exactly L bytes (64 .. 1,024, IB's 1,976) as messages, as contiguous descriptor
    runs (after the census has seen them) and mixed 9:1 with large fragments (4 KiB .. 300 KB) at aligned and odd
    addresses in one descriptor batch, every fragment against the oracle; random registers."""
    import torch

    dv = _dv()
    rng = np.random.default_rng(L * 3 + mode)
    n = 1 << 20 if L <= 256 else 300 * 4096 // L * 2
    base = torch.empty(n * L + (48 << 20), dtype=torch.uint8, device=cuda)
    dv.fill_stream(base, seed=L + 31)
    host = base.cpu().numpy()
    part = int(rng.integers(0, 2**32))
    # the message and its contiguous descriptor run
    got = dv.as_u32(dv.msg_csum(base[:n * L], L, partial=part, mode=mode))
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    lens = np.full(n, L, np.uint32)
    want = oracle.desc_batch(host, offs, lens, np.full(n, part, np.uint32) if mode == 0 else None, mode)
    assert np.array_equal(got, want)
    descs = dv.make_descs(base, offs, lens, np.full(n, part, np.uint64))
    stream = torch.cuda.Stream(device=cuda)
    with torch.cuda.stream(stream):
        for _ in range(3):
            assert np.array_equal(dv.as_u32(dv.frag_csum_batch(descs, mode=mode, stream=stream)), want)
    # mixed with large fragments, aligned and odd addresses
    m = 60000
    big = rng.random(m) < 0.1
    mlens = np.where(big, rng.integers(4096, 300000, size=m), L).astype(np.uint64)
    moffs = rng.integers(0, base.numel() - 300001, size=m).astype(np.uint64)
    moffs[~big & (rng.random(m) < 0.7)] &= ~np.uint64(15)
    parts = rng.integers(0, 2**32, size=m, dtype=np.uint64)
    mdescs = dv.make_descs(base, moffs, mlens, parts)
    mwant = oracle.desc_batch(host, moffs, mlens.astype(np.uint32), parts.astype(np.uint32) if mode == 0 else None,
                              mode)
    assert np.array_equal(dv.as_u32(dv.frag_csum_batch(mdescs, mode=mode)), mwant)


def test_kat_check_values(cuda):
    import torch

    dv = _dv()
    t = torch.tensor(list(b"123456789"), dtype=torch.uint8, device=cuda)
    assert dv.as_u32(dv.msg_csum(t, 4096))[0] == 0x0376E6E7
    assert dv.as_u32(dv.msg_csum(t, 4096, mode=dv.SUM32))[0] == 0x6C6A689F
    z = torch.zeros(65536, dtype=torch.uint8, device=cuda)
    assert dv.as_u32(dv.msg_csum(z, 65536))[0] == 0x288E1614  # uicrc(Z, 65536)
    f = torch.full((4096,), 0xFF, dtype=torch.uint8, device=cuda)
    assert dv.as_u32(dv.msg_csum(f, 4096))[0] == 0xAF19D570
    r = torch.arange(1976, dtype=torch.int32, device=cuda).to(torch.uint8)
    assert dv.as_u32(dv.msg_csum(r, 1976))[0] == 0x092CD62F
    assert dv.as_u32(dv.msg_csum(r, 1976, mode=dv.SUM32))[0] == 0x677786AC


def test_config_b_full_digest(cuda):
    """BASELINE config B: 4M x 4 KiB device-resident; digests from BASELINE.md."""
    import torch

    from oracle.oracle import digest

    dv = _dv()
    n, L = 4194304, 4096
    buf = torch.empty(n * L, dtype=torch.uint8, device=cuda)
    dv.fill_stream(buf, seed=2)
    crc = dv.as_u32(dv.msg_csum(buf, L))
    assert [f"{v:08x}" for v in crc[:4]] == ["9aff1c82", "cf9217cf", "84a13b32", "66922667"]
    assert digest(crc) == (0x959621BB, 0xC38D8899)
    s = dv.as_u32(dv.msg_csum(buf, L, mode=dv.SUM32))
    sx = int(np.sum(s, dtype=np.uint64) & 0xFFFFFFFF)
    assert (sx, digest(s)[1]) == (0x190D78D3, 0x88569035)
    del buf
    torch.cuda.empty_cache()


def test_config_d_shard_digest_sample(cuda, oracle):
    """Config D layout (16 KiB fragments, GPU g owns k = g mod 8): a 1 GiB slice of shard 3."""
    import torch

    dv = _dv()
    n, L, g = 65536, 16384, 3
    buf = torch.empty(n * L, dtype=torch.uint8, device=cuda)
    dv.fill_stream_frags(buf, n, L, seed=3, k0=g, kstep=8)
    got = dv.as_u32(dv.msg_csum(buf, L))
    idx = np.r_[0:256, n - 256:n]
    want = np.array([oracle.uniform_batch(3, g + 8 * int(i), 1, L, 0)[0] for i in idx], dtype=np.uint32)
    assert np.array_equal(got[idx], want)
    if g == 3:
        assert got[0] == oracle.uniform_batch(3, 3, 1, L, 0)[0]


def _bench_digests():
    import json

    with open(os.path.join(os.path.dirname(__file__), "golden", "bench_digests.json")) as f:
        return json.load(f)["entries"]


@pytest.mark.parametrize("g,mode", [(0, "crc"), (7, "crc"), (3, "sum")])
def test_config_d_full_shard_digest(cuda, g, mode):
    """BASELINE config D, GPU g's whole shard of the 8-GPU partition on this one GPU: 4,194,304 x
    16 KiB = 64 GiB (k = g mod 8, seed 3), one lampi_msg_csum launch; XOR and WSUM (global k)
    vs tests/golden/bench_digests.json, and for CRC the XOR vs BASELINE.md's per-GPU value."""
    import torch

    from lampi_amd import shard

    dv = _dv()
    per_gpu_xor = [0x54862C49, 0x046DA633, 0x53ABB493, 0xEB1A2E44, 0xB9EACC67, 0x0BEC3926, 0x937B2402, 0x3B821C43]
    want = [(e["xor"], e["wsum"]) for e in _bench_digests()
            if (e["seed"], e["frag_bytes"], e["mode"], e.get("nshard"), e.get("shard")) == (3, 16384, mode, 8, g)]
    assert len(want) == 1
    if mode == "crc":
        assert want[0][0] == per_gpu_xor[g]
    n, L = 33554432 // 8, 16384
    torch.cuda.empty_cache()
    buf = torch.empty(n * L, dtype=torch.uint8, device=cuda)
    dv.fill_stream_frags(buf, n, L, seed=3, k0=g, kstep=8)
    vals = dv.as_u32(dv.msg_csum(buf, L, mode=dv.CRC32 if mode == "crc" else dv.SUM32))
    del buf
    torch.cuda.empty_cache()
    got = shard.digest(vals, np.arange(n, dtype=np.uint64) * 8 + g)
    assert got == want[0]


def test_host_api_matches_reference_semantics(cuda, oracle):
    """lampi_amd.memfunctions (host entry points, computed on the GPU) vs the oracle."""
    import lampi_amd as la

    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, size=3 << 20, dtype=np.uint8)
    # 8 KiB..256 KiB: the zero-copy sizes (CRC in 4 KiB pieces, SUM in one kernel reading aligned
    # words past the body's end: 262,144 is the largest zero-copy call)
    for n in [0, 1, 3, 4, 5, 100, 4096, 8192, 8193, 65456, 65537, 262143, 262144, 262145, 1 << 20, (3 << 20) - 5]:
        for off in (0, 1, 3):
            src = data[off:off + n]
            p = int(rng.integers(0, 2**32))
            assert la.uicrc(src, n, p) == oracle.uicrc(src, n, p)
            assert la.uicrc(src, n) == oracle.uicrc(src, n)
            for plen in (0, 1, 2, 3):
                pint = int(rng.integers(0, 2**32)) & ((1 << (8 * plen)) - 1)
                st = la.PartialState(pint, plen)
                got = la.uicsum(src, n, st)
                want = oracle.uicsum(src, n, pint, plen)
                assert (got, st.pint, st.plen) == want, (n, off, plen)
    # bcopy with copylen < crclen, = and >
    src = data[:200000]
    for copylen, clen in [(100, 100), (50, 100), (100, 50), (0, 77), (65456, 65456), (70000, 100000)]:
        d1 = np.zeros(200000, np.uint8)
        d2 = np.zeros(200000, np.uint8)
        assert la.bcopy_uicrc(src, d1, copylen, clen) == oracle.bcopy_uicrc(src, d2, copylen, clen)
        assert np.array_equal(d1, d2)
        st = la.PartialState()
        got = la.bcopy_uicsum(src, d1, copylen, clen, st)
        assert (got, st.pint, st.plen) == oracle.bcopy_uicsum(src, d2, copylen, clen)
        assert np.array_equal(d1, d2)


def test_host_bcopy_large_pingpong(cuda, oracle):
    """Host bcopy calls larger than the 8 MiB bounce buffer and not a multiple of its 4 MiB halves:
    the stage-out ping-pong (the halves alternate through events, lampi_csum.cc) for all three
    copy-and-checksum entry points, copylen below, equal to and above the checksum length, source
    and destination at odd offsets.  Destination bytes and checksums vs the oracle."""
    import lampi_amd as la

    rng = np.random.default_rng(91)
    big = (9 << 20) + 13
    data = rng.integers(0, 256, size=big + 4096, dtype=np.uint8)
    for copylen, clen in [(big, big), (big, 5 << 20), ((5 << 20) + 3, big), ((8 << 20) + 1, (8 << 20) + 1)]:
        for soff, doff in [(0, 0), (3, 5)]:
            src = data[soff:soff + max(copylen, clen)]
            d1 = np.full(copylen + doff + 64, 0xA5, np.uint8)
            d2 = d1.copy()
            p = int(rng.integers(0, 2**32))
            got = la.bcopy_uicrc(src, d1[doff:], copylen, clen, p)
            assert got == oracle.bcopy_uicrc(src, d2[doff:], copylen, clen, p), (copylen, clen, soff, doff)
            assert np.array_equal(d1, d2), (copylen, clen, soff, doff)
            d1[:] = 0x5A
            d2[:] = 0x5A
            st = la.PartialState(0x00ABCDEF & 0xFFFF, 2)
            got = la.bcopy_uicsum(src, d1[doff:], copylen, clen, st)
            assert (got, st.pint, st.plen) == oracle.bcopy_uicsum(src, d2[doff:], copylen, clen, 0xCDEF, 2)
            assert np.array_equal(d1, d2), (copylen, clen, soff, doff)
            d1[:] = 0x3C
            d2[:] = 0x3C
            st = la.PartialState64(0x123456, 3)
            got = la.bcopy_csum(src, d1[doff:], copylen, clen, st)
            assert (got, st.plong, st.plen) == oracle.bcopy_csum(src, d2[doff:], copylen, clen, 0x123456, 3)
            assert np.array_equal(d1, d2), (copylen, clen, soff, doff)


def test_host_api_chaining(cuda, oracle):
    """Chained pieces (the non-contiguous typemap pattern, src/path/gm/sendFrag.cc:157-217)."""
    import lampi_amd as la

    rng = np.random.default_rng(3)
    msg = rng.integers(0, 256, size=300000, dtype=np.uint8)
    for _ in range(20):
        cuts = np.sort(rng.integers(0, msg.size, size=int(rng.integers(1, 8))))
        pieces = np.split(msg, cuts)
        crc = la.CRC_INITIAL_REGISTER
        total = 0
        st = la.PartialState()
        for p in pieces:
            crc = la.uicrc(p, p.size, crc)
            total = (total + la.uicsum(p, p.size, st)) & 0xFFFFFFFF
        assert crc == oracle.uicrc(msg)
        assert total == oracle.uicsum(msg)[0]


def test_header_checksum_residue(cuda, oracle):
    """CRC(header || stored headerChecksum) == 0 (receiver check, src/path/gm/path.cc:379-384)."""
    import lampi_amd as la

    rng = np.random.default_rng(8)
    for hl, words in ((72, 18), (128, 32)):
        for _ in range(5):
            hdr = rng.integers(0, 256, size=hl, dtype=np.uint8)
            c = la.header_checksum(hdr, hl - 4, words, usecrc=True)
            assert c == oracle.header_checksum(hdr, hl - 4, words, True)
            hdr[hl - 4:] = np.frombuffer(c.to_bytes(4, "little"), np.uint8)
            assert la.uicrc(hdr, hl) == 0
            assert la.header_checksum(hdr, hl - 4, words, usecrc=False) == oracle.header_checksum(
                hdr, hl - 4, words, False)


def test_config_c_mixed_sizes_full_digest(cuda, oracle):
    """BASELINE config C: 659,114 Zipf-sized fragments (64 B..64 KiB, 4 GiB) as one descriptor
    batch; digest from tests/golden/fixtures.json (restatement, pinned to the reference)."""
    import json
    import os

    import torch

    from oracle.oracle import digest

    dv = _dv()
    with open(os.path.join(os.path.dirname(__file__), "golden", "fixtures.json")) as f:
        gold = json.load(f)["digests"]["C"]
    lens = oracle.zipf_lengths(4 << 30)
    assert lens.size == gold["n"] and int(lens.sum(dtype=np.uint64)) == gold["total_bytes"]
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    buf = torch.empty(gold["total_bytes"], dtype=torch.uint8, device=cuda)
    dv.fill_stream(buf, seed=5)
    descs = dv.make_descs(buf, offs, lens)
    crc = dv.as_u32(dv.frag_csum_batch(descs, mode=dv.CRC32))
    assert [int(v) for v in crc[:4]] == gold["crc_first4"]
    assert digest(crc) == (gold["crc_xor"], gold["crc_wsum"])
    s = dv.as_u32(dv.frag_csum_batch(descs, mode=dv.SUM32))
    assert (int(np.sum(s, dtype=np.uint64) & 0xFFFFFFFF), digest(s)[1]) == (gold["sum_total"], gold["sum_wsum"])
    # the one-wavefront-per-fragment schedule on the same batch (bench.py --config C reports both)
    assert np.array_equal(dv.as_u32(dv.diag_frag_csum_batch_per_wave(descs, mode=dv.CRC32)), crc)
    assert np.array_equal(dv.as_u32(dv.diag_frag_csum_batch_per_wave(descs, mode=dv.SUM32)), s)
    del buf
    torch.cuda.empty_cache()


def test_config_e_message_digests(cuda):
    """BASELINE config E: 256 MiB message (seed 6) fragmented at 4 KiB, 16 KiB and the GM payload size."""
    import json
    import os

    import torch

    from oracle.oracle import digest

    dv = _dv()
    with open(os.path.join(os.path.dirname(__file__), "golden", "fixtures.json")) as f:
        gold = json.load(f)["digests"]["E"]
    msg = torch.empty(256 << 20, dtype=torch.uint8, device=cuda)
    dv.fill_stream(msg, seed=6)
    for L in (4096, 16384, 65456):
        crc = dv.as_u32(dv.msg_csum(msg, L))
        assert crc.size == gold[str(L)]["n"]
        assert digest(crc) == (gold[str(L)]["crc_xor"], gold[str(L)]["crc_wsum"]), L
