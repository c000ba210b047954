#!/usr/bin/env python3
"""Generate tests/golden/fixtures.json from the REFERENCE ITSELF.

The reference's src/util/MemFunctions.cc is compiled unmodified into
oracle/_ref/libref_memfunctions.so (oracle/Makefile, only where /root/reference exists) and
called through its C++ mangled symbols.  Payload bytes are not stored: every case names a
(seed, byte offset, length) slice of the SURVEY.md 8(d) splitmix64 stream, which
oracle.splitmix_stream regenerates, so the fixture stays small.  Digests of the big
BASELINE configs are produced by the restatement (OpenMP) and cross-checked here against
the values BASELINE.md quotes from the survey's oracle probe.

Run:  make -C oracle && python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle.oracle import Reference, Restatement, digest, splitmix_stream  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures.json")

KAT_LENS = [0, 1, 3, 4, 64, 1024, 1976, 4096, 16384, 65456, 65536]
EDGE = [0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 63, 64, 65, 68, 72, 124, 128, 1023, 1024, 1025, 1976, 4095,
        4096, 4097, 16384, 65455, 65456, 65536]


def pattern(kind: str, n: int) -> np.ndarray:
    if kind == "Z":
        return np.zeros(n, np.uint8)
    if kind == "F":
        return np.full(n, 0xFF, np.uint8)
    return (np.arange(n) & 0xFF).astype(np.uint8)


def main():
    ref = Reference()
    port = Restatement()
    rng = random.Random(20261015)
    fx = {"generator": "tests/golden/make_golden.py", "reference": "src/util/MemFunctions.cc (compiled unmodified)",
          "stream": "SURVEY.md 8(d) splitmix64; payload = stream(seed)[off:off+len]"}

    # 1. known answers (SURVEY.md 8(c) table + check strings)
    kat = []
    for n in KAT_LENS:
        row = {"len": n}
        for k in "ZFR":
            buf = pattern(k, n)
            row[f"uicrc_{k}"] = ref.uicrc(buf, n)
            row[f"uicsum_{k}"] = ref.uicsum(buf, n)[0]
        kat.append(row)
    fx["kat"] = kat
    fx["check"] = {"uicrc_123456789": ref.uicrc(b"123456789"), "uicsum_123456789": ref.uicsum(b"123456789")[0]}

    # 2. single calls: random slices, random register / partial-word state
    cases = []
    for i in range(600):
        n = rng.choice(EDGE) if i % 3 == 0 else rng.choice([rng.randrange(0, 300), rng.randrange(0, 70000)])
        seed, off = rng.randrange(1, 1000), rng.randrange(0, 1 << 20)
        buf = splitmix_stream(seed, off, n)
        partial = 0xFFFFFFFF if i % 4 == 0 else rng.getrandbits(32)
        plen = rng.randrange(0, 4)
        pint = rng.getrandbits(8 * plen) if plen else 0
        s, pi2, pl2 = ref.uicsum(buf, n, pint, plen)
        cases.append({"seed": seed, "off": off, "len": n, "partial": partial, "crc": ref.uicrc(buf, n, partial),
                      "pint": pint, "plen": plen, "sum": s, "pint_out": pi2, "plen_out": pl2})
    fx["single"] = cases

    # 3. chained pieces: one message cut into 2-8 pieces (typemap chaining, sendFrag.cc:157-217)
    chains = []
    for _ in range(150):
        n = rng.randrange(0, 20000)
        seed, off = rng.randrange(1, 1000), rng.randrange(0, 1 << 20)
        buf = splitmix_stream(seed, off, n)
        cuts = sorted(rng.randrange(0, n + 1) for _ in range(rng.randrange(1, 8)))
        bounds = [0] + cuts + [n]
        crc, tot, pi, pl = 0xFFFFFFFF, 0, 0, 0
        for a, b in zip(bounds, bounds[1:]):
            crc = ref.uicrc(buf[a:], b - a, crc)
            s, pi, pl = ref.uicsum(buf[a:], b - a, pi, pl)
            tot = (tot + s) & 0xFFFFFFFF
        chains.append({"seed": seed, "off": off, "len": n, "cuts": cuts, "crc": crc, "sum": tot, "pint_out": pi,
                       "plen_out": pl, "crc_whole": ref.uicrc(buf, n), "sum_whole": ref.uicsum(buf, n)[0]})
    fx["chain"] = chains

    # 4. bcopy variants incl. copylen < crclen (receive side, gm/recvFrag.h:174) and src/dst alignment
    bcopy = []
    for i in range(300):
        n = rng.randrange(0, 5000)
        copylen = n if i % 3 == 0 else rng.randrange(0, n + 1)
        clen = n if i % 3 == 1 else rng.randrange(0, n + 1)
        seed, off = rng.randrange(1, 1000), rng.randrange(0, 1 << 20)
        total = max(copylen, clen)
        sa, da = rng.randrange(0, 8), rng.randrange(0, 8)
        src = np.zeros(total + 16, np.uint8)
        src[sa:sa + total] = splitmix_stream(seed, off, total)
        partial = 0xFFFFFFFF if i % 2 else rng.getrandbits(32)
        plen = rng.randrange(0, 4)
        pint = rng.getrandbits(8 * plen) if plen else 0
        d1 = np.zeros(total + 16, np.uint8)
        d2 = np.zeros(total + 16, np.uint8)
        c = ref.bcopy_uicrc(src[sa:], d1[da:], copylen, clen, partial)
        s, pi2, pl2 = ref.bcopy_uicsum(src[sa:], d2[da:], copylen, clen, pint, plen)
        assert np.array_equal(d1[da:da + copylen], src[sa:sa + copylen])
        assert np.array_equal(d2[da:da + copylen], src[sa:sa + copylen])
        bcopy.append({"seed": seed, "off": off, "copylen": copylen, "clen": clen, "src_align": sa, "dst_align": da,
                      "partial": partial, "crc": c, "pint": pint, "plen": plen, "sum": s, "pint_out": pi2,
                      "plen_out": pl2})
    fx["bcopy"] = bcopy

    # 5. alignment independence (MemFunctions.cc aligned / unaligned paths)
    align = []
    for _ in range(40):
        n = rng.randrange(0, 3000)
        seed, off = rng.randrange(1, 1000), rng.randrange(0, 1 << 20)
        body = splitmix_stream(seed, off, n)
        res = []
        for a in range(8):
            b = np.zeros(n + 8, np.uint8)
            b[a:a + n] = body
            res.append([ref.uicrc(b[a:], n), ref.uicsum(b[a:], n)[0]])
        assert all(r == res[0] for r in res)
        align.append({"seed": seed, "off": off, "len": n, "crc": res[0][0], "sum": res[0][1]})
    fx["alignment"] = align

    # 6. digests of the uniform BASELINE configs (restatement, cross-checked with BASELINE.md)
    digs = {}
    t0 = time.time()
    for name, seed, n, L in [("A", 1, 1048576, 1024), ("B", 2, 4194304, 4096)]:
        cx, cw = port.uniform_digest(seed, n, L, 0)
        vals = port.uniform_batch(seed, 0, n, L, 1)
        sx = int(np.sum(vals, dtype=np.uint64) & 0xFFFFFFFF)
        sw = digest(vals)[1]
        first = [int(v) for v in port.uniform_batch(seed, 0, 4, L, 0)]
        digs[name] = {"seed": seed, "n": n, "L": L, "crc_xor": cx, "crc_wsum": cw, "sum_total": sx, "sum_wsum": sw,
                      "crc_first4": first}
    # config A also straight from the reference (1 GiB, single thread)
    a = digs["A"]
    crc_ref = np.empty(a["n"], np.uint32)
    for k0 in range(0, a["n"], 65536):
        blk = splitmix_stream(1, k0 * 1024, 65536 * 1024)
        for i in range(65536):
            crc_ref[k0 + i] = ref.uicrc(blk[i * 1024:(i + 1) * 1024], 1024)
    assert digest(crc_ref) == (a["crc_xor"], a["crc_wsum"]), "restatement digest != reference digest (config A)"
    a["crc_from_reference"] = True
    baseline = {"A": (0xFEB61101, 0x41FADF13, 0xA8714810, 0xC9A787FC),
                "B": (0x959621BB, 0xC38D8899, 0x190D78D3, 0x88569035)}
    for k, v in baseline.items():
        d = digs[k]
        assert (d["crc_xor"], d["crc_wsum"], d["sum_total"], d["sum_wsum"]) == v, f"config {k} != BASELINE.md"
    fx["digests"] = digs
    fx["digests_note"] = ("A: restatement == reference (all 1M fragments); A, B: equal to BASELINE.md; "
                          "D per-GPU shard XORs are BASELINE.md's (not regenerated here)")
    fx["config_d_shard_xor"] = [0x54862C49, 0x046DA633, 0x53ABB493, 0xEB1A2E44, 0xB9EACC67, 0x0BEC3926,
                                0x937B2402, 0x3B821C43]
    # config C (mixed Zipf sizes, seed 5, >= 4 GiB) and config E (256 MiB message, seed 6):
    # restatement-generated (its parity with the reference is pinned by everything above)
    lens = port.zipf_lengths(4 << 30)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.sum(dtype=np.uint64))
    stream = port.stream(5, 0, total)
    crc_c = port.desc_batch(stream, offs, lens, None, 0)
    sum_c = port.desc_batch(stream, offs, lens, None, 1)
    del stream
    cx, cw = digest(crc_c)
    digs["C"] = {"seed": 5, "n": int(lens.size), "total_bytes": total, "crc_xor": cx, "crc_wsum": cw,
                 "sum_total": int(np.sum(sum_c, dtype=np.uint64) & 0xFFFFFFFF), "sum_wsum": digest(sum_c)[1],
                 "len_sum_check": int(lens[:1000].sum()), "crc_first4": [int(v) for v in crc_c[:4]]}
    msg = port.stream(6, 0, 256 << 20)
    digs["E"] = {"seed": 6, "msg_bytes": 256 << 20}
    for L in (4096, 16384, 65456):
        nf = ((256 << 20) + L - 1) // L
        o = np.arange(nf, dtype=np.uint64) * L
        ln = np.minimum(L, (256 << 20) - o).astype(np.uint32)
        v = port.desc_batch(msg, o, ln, None, 0)
        digs["E"][str(L)] = {"n": int(nf), "crc_xor": digest(v)[0], "crc_wsum": digest(v)[1]}
    print(f"digests in {time.time() - t0:.1f}s")

    with open(OUT, "w") as f:
        json.dump(fx, f, separators=(",", ":"))
    print(f"wrote {OUT} ({os.path.getsize(OUT)} bytes)")


if __name__ == "__main__":
    main()
