"""CPU: the C-ABI library builds, loads, and exports exactly what include/lampi_csum.h declares.

No compute calls here (no GPU in this container); the kernels are exercised by -m gpu tests.
"""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "lampi_csum.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lampi_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_drop_in_set():
    names = declared_functions()
    for required in ("lampi_uicrc", "lampi_bcopy_uicrc", "lampi_uicsum", "lampi_bcopy_uicsum",
                     "lampi_frag_csum_batch", "lampi_msg_csum"):
        assert required in names


def test_library_exports_every_declared_symbol():
    import lampi_amd

    lib = lampi_amd.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", lampi_amd._lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (lampi_[a-z0-9_]+)", out))
    for name in declared_functions():
        assert name in exported, name
        assert getattr(lib, name) is not None
    # and the Python prototypes cover the whole C ABI
    assert set(lampi_amd._lib.PROTOTYPES) == set(declared_functions())


def test_library_targets_gfx950():
    """The embedded code object is built for gfx950 (and only for it)."""
    import lampi_amd

    data = open(lampi_amd._lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in data


def test_version_string_needs_no_gpu():
    import lampi_amd

    assert b"gfx950" in lampi_amd.lib().lampi_csum_version()


def test_desc_struct_layout():
    import lampi_amd

    FD = lampi_amd.FragDesc
    assert ctypes.sizeof(FD) == 16
    assert FD.addr.offset == 0 and FD.length.offset == 8 and FD.partial.offset == 12


def test_no_oracle_in_product():
    """The product library and package never reference the oracle (test infrastructure)."""
    import lampi_amd

    out = subprocess.run(["nm", "-D", lampi_amd._lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    assert "oracle_" not in out
    pkg = os.path.join(ROOT, "lampi_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cc", ".hip", ".h")):
                text = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in text and "from oracle" not in text, f
                assert "csum_ref" not in text, f


def test_host_entry_points_fail_loudly_without_gpu():
    """No CPU fallback: without a GPU a host entry point aborts instead of computing."""
    code = ("import sys; sys.path.insert(0, %r); import lampi_amd; "
            "print(lampi_amd.uicrc(b'123456789'))" % ROOT)
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1", CUDA_VISIBLE_DEVICES="-1")
    r = subprocess.run(["python", "-c", code], capture_output=True, text=True, env=env, timeout=120)
    if r.returncode == 0:
        pytest.fail(f"host path returned without a GPU: {r.stdout!r}")
    assert "no CPU fallback" in r.stderr or r.returncode != 0
