"""CPU: the GF(2) tables the kernels stage into LDS reproduce the reference CRC.

tests/native/emulate_rows.cc runs the kernels' exact decomposition (right-aligned 4 KiB-row
frame, lane-contiguous 64-byte pieces, partial injected as data, swapped-domain slicing-by-4,
Horner row shift, per-lane final shift, XOR across lanes) on the table image built by
lampi_amd/csrc/crc_tables.cc, against the byte-serial CRC.
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_row_decomposition_emulation(tmp_path):
    exe = tmp_path / "emulate_rows"
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "emulate_rows.cc"),
                    os.path.join(ROOT, "lampi_amd", "csrc", "crc_tables.cc")], check=True)
    r = subprocess.run([str(exe), "600"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
