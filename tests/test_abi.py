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


# the reference's twelve overloads (src/util/MemFunctions.h:43-65) by their mangled names
REFERENCE_MANGLED = [
    "_Z5uicrcPKvm", "_Z5uicrcPKvmj", "_Z11bcopy_uicrcPKvPvmm", "_Z11bcopy_uicrcPKvPvmmj",
    "_Z6uicsumPKvm", "_Z6uicsumPKvmPjS1_", "_Z12bcopy_uicsumPKvPvmm", "_Z12bcopy_uicsumPKvPvmmPjS2_",
    "_Z4csumPKvm", "_Z4csumPKvmPmS1_", "_Z10bcopy_csumPKvPvmm", "_Z10bcopy_csumPKvPvmmPmS2_",
    # the rest of MemFunctions.o (MemFunctions.cc:1242-1261, :1380-1393)
    "_Z24ulm_initialize_crc_tablev", "_Z12poisonMemoryPvli",
]


def test_library_exports_the_reference_cxx_abi():
    """libmpi can swap MemFunctions.o for -llampi_csum without recompiling: the library defines every
    function of the reference's object (the twelve overloads, ulm_initialize_crc_table, poisonMemory)
    under its mangled name -- exactly the set the compiled reference exports."""
    import lampi_amd

    out = subprocess.run(["nm", "-D", "--defined-only", lampi_amd._lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (_Z\w+)", out))
    for name in REFERENCE_MANGLED:
        assert name in exported, name
    ref = os.path.join(ROOT, "oracle", "_ref", "libref_memfunctions.so")
    if os.path.exists(ref):  # the reference compiled here exports exactly these
        rout = subprocess.run(["nm", "-D", "--defined-only", ref], capture_output=True, text=True, check=True).stdout
        assert set(re.findall(r" T (_Z\w+)", rout)) == set(REFERENCE_MANGLED)


def test_object_compiled_against_reference_header_links(tmp_path):
    """A caller compiled against the REFERENCE's own MemFunctions.h (this container only) links against
    liblampi_csum.so alone: a relink, no source or header change."""
    import lampi_amd

    ref_src = "/root/reference/src"
    if not os.path.exists(os.path.join(ref_src, "util", "MemFunctions.h")):
        pytest.skip("reference sources absent")
    src = tmp_path / "ref_caller.cc"
    src.write_text(r'''
#include "util/MemFunctions.h"
unsigned int f(const void *s, void *d, unsigned long n) {
    unsigned int a = 0, b = 0;
    unsigned long c = 0, e = 0;
    return uicrc(s, n) + uicrc(s, n, 1u) + bcopy_uicrc(s, d, n, n) + bcopy_uicrc(s, d, n, n, 1u) + uicsum(s, n) +
           uicsum(s, n, &a, &b) + bcopy_uicsum(s, d, n, n) + bcopy_uicsum(s, d, n, n, &a, &b) +
           (unsigned)(csum(s, n) + csum(s, n, &c, &e) + bcopy_csum(s, d, n, n) + bcopy_csum(s, d, n, n, &c, &e));
}
void poisonMemory(void *ptr, ssize_t lenInBytes, int pattern);  // src/util/Utility.h:45
void ulm_initialize_crc_table();                                  // MemFunctions.cc:1242
void g(void *p) { ulm_initialize_crc_table(); poisonMemory(p, 64, 0x5a5a5a5a); }
int main(int argc, char **) { return argc > 5 ? (int)f(0, 0, 0) : 0; }
''')
    libdir = os.path.dirname(lampi_amd._lib.LIB_PATH)
    subprocess.run(["g++", "-w", "-I", ref_src, "-I", os.path.join(ref_src, "include"), str(src), "-L", libdir,
                    "-llampi_csum", "-o", str(tmp_path / "ref_caller")], check=True)


def test_library_targets_gfx950():
    """The embedded code object is built for gfx950 (and only for it)."""
    import lampi_amd

    data = open(lampi_amd._lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in data


def _kernel_metadata():
    """(name, private_segment_fixed_size, vgpr_count) of every kernel in the library's gfx950 code
    object (offload bundle entry -> llvm-readelf --notes)."""
    import re
    import struct
    import tempfile

    import lampi_amd

    data = open(lampi_amd._lib.LIB_PATH, "rb").read()
    i = data.find(b"__CLANG_OFFLOAD_BUNDLE__")
    assert i >= 0, "no offload bundle in the library"
    n = struct.unpack_from("<Q", data, i + 24)[0]
    p, co = i + 32, None
    for _ in range(n):
        off, size, ts = struct.unpack_from("<QQQ", data, p)
        p += 24
        triple = data[p:p + ts]
        p += ts
        if b"gfx950" in triple:
            co = data[i + off:i + off + size]
    assert co, "no gfx950 entry in the offload bundle"
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", f.name], capture_output=True,
                             text=True, check=True).stdout
    kernels = []
    for e in re.split(r"\n  - \.agpr_count", out[out.find(".kernels:"):])[1:]:
        kernels.append((re.search(r"\n    \.name:\s+(\S+)", e).group(1),
                        int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", e).group(1)),
                        int(re.search(r"\.vgpr_count:\s+(\d+)", e).group(1))))
    return kernels


def test_kernels_use_no_scratch():
    """No kernel spills to scratch.  The row kernels issue their loads by inline asm and wait for
    them with explicit vmcnt: a spill of a register that an asm load is still writing reads
    garbage (a 64-VGPR experiment of the regular kernel that spilled faulted on the GPU).  The
    stream kernel must also stay within 80 VGPRs (six waves per SIMD: the occupancy it was
    measured at)."""
    ks = _kernel_metadata()
    assert len(ks) >= 20
    assert [k for k in ks if k[1] != 0] == []
    stream = [k for k in ks if "crc_stream_kernel" in k[0]]
    assert stream and all(k[2] <= 80 for k in stream), stream


def test_version_string_needs_no_gpu():
    import lampi_amd

    assert b"gfx950" in lampi_amd.lib().lampi_csum_version()


def test_desc_struct_layout():
    import lampi_amd

    FD = lampi_amd.FragDesc
    assert ctypes.sizeof(FD) == 16
    assert FD.addr.offset == 0 and FD.length.offset == 8 and FD.partial.offset == 12
    CD = lampi_amd._lib.CopyDesc
    assert ctypes.sizeof(CD) == 32
    assert [getattr(CD, f).offset for f in ("src", "dst", "copylen", "csumlen", "partial", "reserved")] == \
        [0, 8, 16, 20, 24, 28]


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


def test_reference_callers_compile_against_dropin_header(tmp_path):
    """Code written against the reference's MemFunctions.h overloads compiles and links
    against include/lampi/MemFunctions.h + liblampi_csum.so."""
    import lampi_amd

    src = tmp_path / "caller.cc"
    src.write_text(r'''
#include "lampi/MemFunctions.h"
// the shapes of the src/path call sites (gm/sendFrag.cc:147-217, gm/recvFrag.h:165-182)
unsigned int send_contig(const void *s, void *d, unsigned long n) { return bcopy_uicrc(s, d, n, n); }
unsigned int send_typemap(const void *s, void *d, unsigned long n) {
    unsigned int csum = 0, ui1 = 0, ui2 = 0;
    csum = bcopy_uicrc(s, d, n, n, CRC_INITIAL_REGISTER);
    csum += bcopy_uicsum(s, d, n, n, &ui1, &ui2);
    return csum + uicsum(s, n) + uicsum(s, n, &ui1, &ui2) + uicrc(s, n) + uicrc(s, n, csum) +
           bcopy_uicsum(s, d, n, n);
}
unsigned long sum64(const void *s, void *d, unsigned long n) {  // MemFunctions.h:43-50 overloads
    unsigned long pl = 0, pn = 0;
    return csum(s, n) + csum(s, n, &pl, &pn) + bcopy_csum(s, d, n, n) + bcopy_csum(s, d, n, n, &pl, &pn);
}
int main(int argc, char **) { return argc > 5 ? (int)(send_contig(0, 0, 0) + sum64(0, 0, 0)) : 0; }
''')
    c_src = tmp_path / "caller.c"
    c_src.write_text(r'''
#include "lampi_csum.h"
int main(void) {
    lampi_frag_desc d = {0, 0, LAMPI_CRC_INITIAL_REGISTER};
    (void)d;
    lampi_copy_desc c = {0, 0, 0, 0, LAMPI_CRC_INITIAL_REGISTER, 0};
    (void)c;
    return (int)(sizeof(lampi_frag_desc) != 16 || sizeof(lampi_copy_desc) != 32);
}
''')
    libdir = os.path.dirname(lampi_amd._lib.LIB_PATH)
    inc = os.path.join(ROOT, "include")
    subprocess.run(["g++", "-std=c++11", "-Wall", "-Werror", "-I", inc, str(src), "-L", libdir, "-llampi_csum",
                    "-o", str(tmp_path / "caller")], check=True)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", inc, str(c_src), "-o", str(tmp_path / "cc")],
                   check=True)
    assert subprocess.run([str(tmp_path / "cc")]).returncode == 0


def test_mode_flag_macros_match_the_binding(tmp_path):
    """The header's mode flags (LAMPI_CSUM_BY_BYTES, LAMPI_CSUM_ROWS_HINT) as a C caller sees them equal
    what the Python binding ORs into `mode`, and the hint field does not overlap the mode or BY_BYTES."""
    from lampi_amd._lib import BY_BYTES, CRC32, SUM32, rows_hint_bits

    prog = tmp_path / "flags.c"
    prog.write_text('#include "lampi_csum.h"\n#include <stdio.h>\n'
                    'int main(void) { printf("%d %d %u %u %u\\n", LAMPI_CSUM_BY_BYTES, LAMPI_CSUM_ROWS_HINT(16), '
                    'LAMPI_CSUM_ROWS_HINT_OF(LAMPI_CSUM_ROWS_HINT(4095) | LAMPI_CSUM_BY_BYTES | 1), '
                    '(unsigned)LAMPI_CSUM_ROWS_HINT_MASK, LAMPI_CSUM_ROWS_HINT_OF(-1)); return 0; }\n')
    exe = tmp_path / "flags"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.dirname(HEADER), str(prog), "-o", str(exe)],
                   check=True)
    by_bytes, hint16, back, mask, of_all = (int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True,
                                                                           text=True).stdout.split())
    assert by_bytes == BY_BYTES and hint16 == rows_hint_bits(16) and back == 4095
    assert mask & (BY_BYTES | CRC32 | SUM32) == 0 and of_all == 4095
    with pytest.raises(ValueError):
        rows_hint_bits(4096)


def test_default_library_reads_no_ab_knobs():
    """the schedule knobs measured in A/B runs are compiled only into the A/B build
    (make AB=1 -> liblampi_csum_ab.so, LAMPI_AB_KNOBS); the default library's dispatch depends on no
    environment variable but the documented switches (LAMPI_CSUM_NO_SHAPES, LAMPI_HOST_CHUNK_BYTES) -- none of
    the knob names is in its binary, and every getenv in the sources goes through LAMPI_AB_ENV or is documented."""
    csrc = os.path.join(ROOT, "lampi_amd", "csrc")
    knobs, documented = set(), {"LAMPI_CSUM_NO_SHAPES", "LAMPI_HOST_CHUNK_BYTES"}
    for name in os.listdir(csrc):
        if not name.endswith((".hip", ".cc", ".h")):
            continue
        src = open(os.path.join(csrc, name)).read()
        knobs |= set(re.findall(r'LAMPI_AB_ENV\("([A-Z0-9_]+)"\)', src))
        direct = set(re.findall(r'getenv\("([A-Z0-9_]+)"\)', src))
        assert direct <= documented, (name, direct - documented)
    assert len(knobs) >= 20, knobs
    import lampi_amd

    blob = open(lampi_amd._lib.LIB_PATH, "rb").read()
    present = sorted(k for k in knobs if k.encode() in blob)
    assert not present, present
    for k in documented:
        assert k.encode() in blob, k
