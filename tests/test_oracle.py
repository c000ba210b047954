"""CPU: the oracle restatement is pinned to the reference.

* against the committed fixtures generated from the compiled reference (tests/golden/);
* against the SURVEY.md 8(c) known-answer table and BASELINE.md digests;
* against the reference itself (oracle/_ref) on fresh random cases, where it is built.
"""
import json
import os

import numpy as np
import pytest

from oracle.oracle import digest, splitmix_stream

FIX = os.path.join(os.path.dirname(__file__), "golden", "fixtures.json")


@pytest.fixture(scope="module")
def fx():
    with open(FIX) as f:
        return json.load(f)


# len -> (uicrc Z, uicrc F, uicrc R, uicsum F, uicsum R)
SURVEY_KAT = {
    0: (0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0x00000000, 0x00000000),
    1: (0x4E08BFB4, 0xFFFFFF00, 0x4E08BFB4, 0x000000FF, 0x00000000),
    3: (0xB7647D00, 0xFF000000, 0x6CFF87B2, 0x00FFFFFF, 0x00020100),
    4: (0xC704DD7B, 0x00000000, 0x6B6DC92A, 0xFFFFFFFF, 0x03020100),
    64: (0x93394E51, 0xA21E790F, 0xBCBD08F5, 0xFFFFFFF0, 0x1201F1E0),
    1024: (0x8B0A5208, 0xD000A3E2, 0x1A5C3E13, 0xFFFFFF00, 0x807F7E00),
    1976: (0xCB7F3544, 0xC538F888, 0x092CD62F, 0xFFFFFE12, 0x677786AC),
    4096: (0x77FFC71C, 0xAF19D570, 0x35062FD6, 0xFFFFFC00, 0x01FDF800),
    16384: (0x9EB4D52A, 0x34132F69, 0x2BDE5F51, 0xFFFFF000, 0x07F7E000),
    65456: (0x850E24B5, 0xAE5B1883, 0x2DE4FFE4, 0xFFFFC014, 0x1AEEA348),
    65536: (0x288E1614, 0x8D812A84, 0xD4918705, 0xFFFFC000, 0x1FDF8000),
}


def _pat(k, n):
    if k == "Z":
        return np.zeros(n, np.uint8)
    if k == "F":
        return np.full(n, 0xFF, np.uint8)
    return (np.arange(n) & 0xFF).astype(np.uint8)


def test_survey_kat_table(oracle):
    for n, (cz, cf, cr, sf, sr) in SURVEY_KAT.items():
        assert oracle.uicrc(_pat("Z", n), n) == cz
        assert oracle.uicrc(_pat("F", n), n) == cf
        assert oracle.uicrc(_pat("R", n), n) == cr
        assert oracle.uicsum(_pat("F", n), n)[0] == sf
        assert oracle.uicsum(_pat("R", n), n)[0] == sr
        assert oracle.uicsum(_pat("Z", n), n)[0] == 0
    assert oracle.uicrc(b"123456789") == 0x0376E6E7  # CRC-32/MPEG-2 check value
    assert oracle.uicsum(b"123456789")[0] == 0x6C6A689F


def test_fixture_kat(oracle, fx):
    for row in fx["kat"]:
        n = row["len"]
        for k in "ZFR":
            assert oracle.uicrc(_pat(k, n), n) == row[f"uicrc_{k}"]
            assert oracle.uicsum(_pat(k, n), n)[0] == row[f"uicsum_{k}"]
        assert (row["uicrc_Z"], row["uicrc_F"], row["uicrc_R"], row["uicsum_F"], row["uicsum_R"]) == SURVEY_KAT[n]
    assert fx["check"]["uicrc_123456789"] == 0x0376E6E7


def test_fixture_single(oracle, fx):
    for c in fx["single"]:
        buf = splitmix_stream(c["seed"], c["off"], c["len"])
        assert oracle.uicrc(buf, c["len"], c["partial"]) == c["crc"]
        assert oracle.uicsum(buf, c["len"], c["pint"], c["plen"]) == (c["sum"], c["pint_out"], c["plen_out"])


def test_fixture_chain(oracle, fx):
    for c in fx["chain"]:
        buf = splitmix_stream(c["seed"], c["off"], c["len"])
        b = [0] + c["cuts"] + [c["len"]]
        crc, tot, pi, pl = 0xFFFFFFFF, 0, 0, 0
        for lo, hi in zip(b, b[1:]):
            crc = oracle.uicrc(buf[lo:], hi - lo, crc)
            s, pi, pl = oracle.uicsum(buf[lo:], hi - lo, pi, pl)
            tot = (tot + s) & 0xFFFFFFFF
        assert (crc, tot, pi, pl) == (c["crc"], c["sum"], c["pint_out"], c["plen_out"])
        assert crc == c["crc_whole"] and tot == c["sum_whole"]  # chaining == whole message


def test_fixture_bcopy(oracle, fx):
    for c in fx["bcopy"]:
        total = max(c["copylen"], c["clen"])
        src = np.zeros(total + 16, np.uint8)
        sa, da = c["src_align"], c["dst_align"]
        src[sa:sa + total] = splitmix_stream(c["seed"], c["off"], total)
        d = np.zeros(total + 16, np.uint8)
        assert oracle.bcopy_uicrc(src[sa:], d[da:], c["copylen"], c["clen"], c["partial"]) == c["crc"]
        assert np.array_equal(d[da:da + c["copylen"]], src[sa:sa + c["copylen"]])
        assert not d[da + c["copylen"]:].any()  # residue bytes are CRC'd, not copied
        d[:] = 0
        got = oracle.bcopy_uicsum(src[sa:], d[da:], c["copylen"], c["clen"], c["pint"], c["plen"])
        assert got == (c["sum"], c["pint_out"], c["plen_out"])


def test_fixture_alignment(oracle, fx):
    for c in fx["alignment"]:
        body = splitmix_stream(c["seed"], c["off"], c["len"])
        for a in range(8):
            b = np.zeros(c["len"] + 8, np.uint8)
            b[a:a + c["len"]] = body
            assert oracle.uicrc(b[a:], c["len"]) == c["crc"]
            assert oracle.uicsum(b[a:], c["len"])[0] == c["sum"]


def test_digest_config_a(oracle, fx):
    d = fx["digests"]["A"]
    assert oracle.uniform_digest(1, d["n"], d["L"], 0) == (0xFEB61101, 0x41FADF13)
    vals = oracle.uniform_batch(1, 0, d["n"], d["L"], 1)
    assert int(np.sum(vals, dtype=np.uint64) & 0xFFFFFFFF) == 0xA8714810
    assert digest(vals)[1] == 0xC9A787FC
    assert [int(v) for v in oracle.uniform_batch(1, 0, 4, 1024, 0)] == [0x24617188, 0x2A607FC5, 0xAB3F43DF,
                                                                       0x477F8C7B]


def test_digest_config_b_and_d_heads(oracle, fx):
    assert [int(v) for v in oracle.uniform_batch(2, 0, 4, 4096, 0)] == [0x9AFF1C82, 0xCF9217CF, 0x84A13B32,
                                                                       0x66922667]
    assert [int(v) for v in oracle.uniform_batch(3, 0, 4, 16384, 0)] == [0x40A5F6EC, 0xCDDC3E91, 0x4580D0EA,
                                                                        0x9B085072]
    d = fx["digests"]["B"]
    assert (d["crc_xor"], d["crc_wsum"], d["sum_total"], d["sum_wsum"]) == (0x959621BB, 0xC38D8899, 0x190D78D3,
                                                                            0x88569035)
    shard = fx["config_d_shard_xor"]
    x = 0
    for v in shard:
        x ^= v
    assert x == 0xF2A5DDAD  # per-GPU shard XORs combine to the config D total


def test_stream_generators_agree(oracle):
    for seed, off, n in [(1, 0, 1000), (2, 3, 4097), (9, 12345, 77)]:
        assert np.array_equal(oracle.stream(seed, off, n), splitmix_stream(seed, off, n))


def test_restatement_vs_reference_fuzz(oracle, reference):
    rng = np.random.default_rng(42)
    buf = rng.integers(0, 256, size=100000, dtype=np.uint8)
    for _ in range(3000):
        off = int(rng.integers(0, 16))
        n = int(rng.choice([rng.integers(0, 10), rng.integers(0, 500), rng.integers(0, 70000)]))
        src = buf[off:off + n]
        p = int(rng.integers(0, 2**32))
        assert oracle.uicrc(src, n, p) == reference.uicrc(src, n, p)
        plen = int(rng.integers(0, 4))
        pint = int(rng.integers(0, 2**32))
        assert oracle.uicsum(src, n, pint, plen) == reference.uicsum(src, n, pint, plen)
        cl, ml = int(rng.integers(0, n + 1)), int(rng.integers(0, n + 1))
        d1, d2 = np.zeros(n + 8, np.uint8), np.zeros(n + 8, np.uint8)
        assert oracle.bcopy_uicrc(src, d1, cl, ml, p) == reference.bcopy_uicrc(src, d2, cl, ml, p)
        assert oracle.bcopy_uicsum(src, d1, cl, ml, pint, plen) == reference.bcopy_uicsum(src, d2, cl, ml, pint,
                                                                                           plen)
        assert np.array_equal(d1, d2)


def test_cpu_baseline_speed_matches_reference(oracle, reference):
    """The restatement is the same byte-serial algorithm: per-core speed within +-20%."""
    buf = oracle.stream(1, 0, 16 << 20)
    # (interleaved, best of seven each: a loaded machine -- pytest -n -- slows both alike)
    tp, tr = float("inf"), float("inf")
    for _ in range(7):
        tp = min(tp, oracle.time_crc_fn(oracle.uicrc_addr(), buf, 16384, 1024, 1)[0])
        tr = min(tr, oracle.time_crc_fn(reference.uicrc_addr(), buf, 16384, 1024, 1)[0])
    assert 0.8 < tp / tr < 1.25, (tp, tr)


def test_csum64_fixtures(oracle):
    """64-bit csum / bcopy_csum restatement vs the reference's own results (tests/golden/csum64.json)."""
    from oracle.oracle import splitmix_stream

    with open(os.path.join(os.path.dirname(__file__), "golden", "csum64.json")) as f:
        g = json.load(f)
    for c in g["single"]:
        got = oracle.csum(splitmix_stream(c["seed"], c["off"], c["len"]), c["len"], c["plong"], c["plen"])
        assert got == (c["sum"], c["plong_out"], c["plen_out"])
    for c in g["chain"]:
        buf = splitmix_stream(c["seed"], c["off"], c["len"])
        bounds = [0] + c["cuts"] + [c["len"]]
        tot, pl, pn = 0, 0, 0
        for a, b in zip(bounds, bounds[1:]):
            s, pl, pn = oracle.csum(buf[a:], b - a, pl, pn)
            tot = (tot + s) % 2**64
        assert tot == c["sum"] == c["sum_whole"]
    for c in g["bcopy"]:
        total = max(c["copylen"], c["clen"])
        src = np.zeros(total + 16, np.uint8)
        src[c["src_align"]:c["src_align"] + total] = splitmix_stream(c["seed"], c["off"], total)
        dst = np.zeros(total + 16, np.uint8)
        got = oracle.bcopy_csum(src[c["src_align"]:], dst[c["dst_align"]:], c["copylen"], c["clen"], c["plong"],
                                c["plen"])
        assert got == (c["sum"], c["plong_out"], c["plen_out"])
        assert np.array_equal(dst[c["dst_align"]:c["dst_align"] + c["copylen"]],
                              src[c["src_align"]:c["src_align"] + c["copylen"]])
