"""GPU: native C++ programs through the drop-in boundary (VERDICT r1 "next" #8).

* tests/native/dropin_caller -- written against the reference's MemFunctions.h overloads
  (ref src/util/MemFunctions.h:43-65), compiled against include/lampi/MemFunctions.h and linked to
  liblampi_csum.so exactly as INTEGRATION.md section 1 tells a maintainer; it runs the src/path
  call shapes (uicrc over a DMA source, bcopy_uicrc with copylen < crclen, chained uicsum state,
  the 64-bit overloads) on four threads and on the main thread around lampi_host_release().
  Every printed result is recomputed here with the oracle (reference-pinned restatement).
* tests/native/host_leak -- 1,000 short-lived threads making host calls (thread-exit release of
  the staging context) and 1,000 call + lampi_host_release() rounds (the release a device switch
  runs): device memory in use must not grow.
Both binaries are built on the CPU by __graft_entry__.build() (make -C tests/native).
"""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _bin(name):
    p = os.path.join(HERE, "native", name)
    if not os.path.exists(p):
        pytest.fail(f"{p} not built: run __graft_entry__.build() (make -C tests/native)")
    return p


def test_native_dropin_caller_matches_oracle(cuda, oracle):
    seed = 11
    r = subprocess.run([_bin("dropin_caller"), str(seed), "4"], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if "->" in ln]
    assert r.stdout.strip().endswith("done")
    buf = oracle.stream(seed, 0, 3 << 20)
    seen = set()
    for ln in lines:
        lhs, rhs = ln.split("->")
        tid, op, off, doff, copylen, csumlen, partial, pint, plen = lhs.split()
        off, copylen, csumlen, partial, pint, plen = map(int, (off, copylen, csumlen, partial, pint, plen))
        res, pi_out, pl_out, ok = map(int, rhs.split())
        src = buf[off:off + max(copylen, csumlen)]
        dst = np.zeros(max(copylen, 1), np.uint8)
        if op == "uicrc":
            want = (oracle.uicrc(src, csumlen),)
        elif op == "uicrc_p":
            want = (oracle.uicrc(src, csumlen, partial),)
        elif op == "bcopy_uicrc":
            want = (oracle.bcopy_uicrc(src, dst, copylen, csumlen),)
        elif op == "bcopy_uicrc_p":
            want = (oracle.bcopy_uicrc(src, dst, copylen, csumlen, partial),)
        elif op == "uicsum":
            want = (oracle.uicsum(src, csumlen)[0],)
        elif op == "uicsum_s":
            want = oracle.uicsum(src, csumlen, pint, plen)
        elif op == "bcopy_uicsum":
            want = (oracle.bcopy_uicsum(src, dst, copylen, csumlen)[0],)
        elif op == "bcopy_uicsum_s":
            want = oracle.bcopy_uicsum(src, dst, copylen, csumlen, pint, plen)
        elif op == "csum":
            want = (oracle.csum(src, csumlen)[0],)
        elif op == "bcopy_csum":
            want = (oracle.bcopy_csum(src, dst, copylen, csumlen)[0],)
        else:
            raise AssertionError(op)
        got = (res, pi_out, pl_out) if len(want) == 3 else (res,)
        assert got == tuple(want), ln
        assert ok == 1, ln
        seen.add((tid, op))
    assert len({t for t, _ in seen}) == 5  # four worker threads + the main thread
    assert len(lines) == (4 + 2) * 16 * 10  # (4 worker threads + 2 main-thread rounds) x 16 cases x 10 ops


def test_native_host_staging_does_not_leak(cuda):
    r = subprocess.run([_bin("host_leak"), "1000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    f = dict(zip(r.stdout.split()[0::2], map(int, r.stdout.split()[1::2])))
    assert f["rounds"] == 1000 and f["bad"] == 0
    # a leaked context holds >= 1 MiB of device buffers: 1,000 leaks would be >= 1 GiB
    assert f["after_threads"] - f["used_before"] < (64 << 20), r.stdout
    assert f["after_release"] - f["used_before"] < (64 << 20), r.stdout
    # page-locked host staging (bounce buffers, result words): exactly back where it was after the
    # thread churn, and none at all once the last context was released
    assert f["pinned_before"] > 0
    assert f["pinned_after_threads"] == f["pinned_before"], r.stdout
    assert f["pinned_after_release"] == 0, r.stdout
    # per-thread device scratch (row-group joins of the receive path): gone with each thread, and
    # after the main thread's release (it was kept per stream until process exit)
    assert f["scratch_after_threads"] == 0 and f["scratch_after_release"] == 0, r.stdout


def test_native_host_message_path_matches_oracle(cuda):
    """lampi_host_msg_csum / lampi_host_msg_bcopy from a native C++ caller (tests/native/host_msg_caller.cc):
    GM 65,456-byte payloads in 64 KiB buffers, 4 KiB / 16 KiB / IB 1,976-byte fragments, a fragment
    larger than a pipeline chunk, short and empty messages, fragment sub-ranges, pinned and pageable
    sources and rings, both modes, two threads at once; every fragment against the oracle inside the
    program, every slot byte against the source, sentinels around the slots untouched."""
    r = subprocess.run([_bin("host_msg_caller"), "6", "2"], capture_output=True, text=True, timeout=600)
    out = r.stdout
    assert r.returncode == 0, out[-4000:] + r.stderr[-2000:]
    assert out.strip().endswith("bad 0 done"), out[-2000:]
    lines = [ln for ln in out.splitlines() if ln.startswith(("csum ", "bcopy_", "invalid"))]
    assert lines and all(ln.endswith(" ok") for ln in lines)
    # 7 shapes x 2 modes x 2 sources x 4 ranges x 3 calls, on 2 threads + the main thread, + 1
    assert len(lines) == 7 * 2 * 2 * 4 * 3 * (2 + 1) + 1
    assert "pinned_after_release 0" in out


def test_native_host_receive_path_matches_oracle(cuda):
    """lampi_host_header_check_batch / _compare_batch and lampi_host_copy_to_app_batch from a native C++
    caller (tests/native/host_recv_caller.cc): GM rings of 64 KiB buffers with 65,456-byte and 4 KiB
    payloads, IB rings of 2,048-byte buffers behind a 40-byte GRH; ~1% corrupted headers (incl. the
    reference's |= 0xA4A4), ~2% corrupted data checksums, ~1% corrupted payloads; AppBufferLen <= 0 / < /
    = / >; ragged and empty fragments; ring-order and shuffled batches; pinned and pageable rings; CRC, SUM
    and checksumming off (LAMPI_CSUM_NONE, headers checked in CRC); two threads at once, then the main thread.  Every verdict, checksum, copied count and
    application byte is checked against the oracle inside the program."""
    r = subprocess.run([_bin("host_recv_caller"), "2"], capture_output=True, text=True, timeout=600)
    out = r.stdout
    assert r.returncode == 0, out[-4000:] + r.stderr[-2000:]
    assert out.strip().endswith("bad 0 done"), out[-2000:]
    lines = [ln for ln in out.splitlines() if ln.startswith(("headers ", "copy_to_app ", "invalid", "empty",
                                                                "nothing"))]
    assert lines and all(ln.endswith(" ok") for ln in lines)
    # 3 shapes x 3 delivery modes (CRC, SUM, checksumming off) x 2 rings x 2 orders x (headers + copy) on 2
    # threads + main, + 4 edge lines
    assert len(lines) == 3 * 3 * 2 * 2 * 2 * (2 + 1) + 4
    # the batches really held corrupt fragments of every kind
    assert any(" nbad 0 " not in ln and ln.startswith("headers ") for ln in lines)
    assert any(ln.startswith("copy_to_app ") and " nbad 0 " not in ln for ln in lines)
    assert "pinned_after_release 0 scratch_after_release 0" in out


def test_native_host_typemap_chains_match_reference(cuda, tmp_path):
    """lampi_host_chain_csum_batch from a native C++ caller (tests/native/host_chain_caller.cc): the
    reference's 150 chain fixtures (values computed by the compiled MemFunctions.cc, passed to the program
    as text), strided-vector typemaps gathered and scattered (8 B .. 4 KiB elements), random typemaps with
    checksum-only and csumlen > copylen pieces and CRC starting registers; both modes, pinned and pageable
    buffers, two threads at once, then the main thread.  Every checksum and destination byte is checked.
    Then lampi_host_chain_copy_to_app_batch (CopyToApp's non-contiguous branch, ref BaseDesc.cc:72-163,
    :326-340): random received fragments scattered into typemap pieces, ~25% corrupted expected values,
    fragments without pieces, CRC / SUM / checksumming off -- every verdict, checksum and byte."""
    import json

    with open(os.path.join(HERE, "golden", "fixtures.json")) as f:
        cases = json.load(f)["chain"]
    path = tmp_path / "chain_cases.txt"
    with open(path, "w") as f:
        for c in cases:
            f.write(" ".join(str(v) for v in [c["seed"], c["off"], c["len"], c["crc"], c["sum"], len(c["cuts"])]
                             + list(c["cuts"])) + "\n")
    r = subprocess.run([_bin("host_chain_caller"), str(path), "2"], capture_output=True, text=True, timeout=600)
    out = r.stdout
    assert r.returncode == 0, out[-4000:] + r.stderr[-2000:]
    assert out.strip().endswith("bad 0 done"), out[-2000:]
    assert f"fixture_cases {len(cases)}" in out and len(cases) == 150
    lines = [ln for ln in out.splitlines()
             if ln.startswith(("fixtures ", "vector_", "random ", "invalid", "fragments", "deliver"))]
    assert lines and all(ln.endswith(" ok") for ln in lines)
    # per thread: 2 x 2 fixture batches, 6 shapes x 2 buffers x 2 modes x (gather + scatter), 6 x 2 random,
    # 4 x 3 deliveries; + 3 edge lines
    assert len(lines) == 3 * (4 + 6 * 2 * 2 * 2 + 6 * 2 + 4 * 3) + 3
    assert any(ln.startswith("deliver ") and " bad 0 " not in ln for ln in lines)
    assert "pinned_after_release 0 scratch_after_release 0" in out


def test_native_send_ring_in_place_matches_oracle(cuda):
    """The device-resident send step in place from a native C++ caller (tests/native/send_ring_caller.cc): a GM
    ring of 64 KiB buffers packed by lampi_msg_bcopy_strided (a message of 65,456-byte fragments),
    lampi_chain_csum_batch_strided (typemap fragments) and lampi_frag_bcopy_batch_strided (ragged descriptors),
    each stamping dataChecksum @64, then lampi_header_csum_batch_strided stamping the header checksum @68
    (ref src/path/gm/sendFrag.cc:143-226) -- CRC, SUM and checksumming off; every byte of the ring against the
    oracle's send loop and the receiver's header test inside the program."""
    r = subprocess.run([_bin("send_ring_caller")], capture_output=True, text=True, timeout=300)
    out = r.stdout
    assert r.returncode == 0, out[-4000:] + r.stderr[-2000:]
    assert out.strip().endswith("bad 0 done"), out[-2000:]
    lines = [ln for ln in out.splitlines() if ln.startswith("send_ring ")]
    assert len(lines) == 3 and all(ln.endswith(" ok") for ln in lines), out
