"""CPU: the asm-issued load rings are safe in the compiler's final code (VERDICT r1 "next" #7).

tests/isa_check.py walks every control-flow path of every kernel in the device assembly of
frag_csum.hip (built with the library's flags by lampi_amd/csrc/Makefile) and fails if any
instruction reads, copies or overwrites the destination registers of an asm-issued load before
the asm wait that names them (or a full vmcnt(0)).  tools/isa_guard/broken_ring.hip holds the
two round-1 failure shapes on purpose -- a copy of an in-flight load, and a ring waited by two
asm statements on two branches (the pre-fix wait selection) -- and round 4's ring drain (a refill
skipped under a branch, its wait chosen on two branches); all must be flagged.
"""
import os
import subprocess

import pytest

import isa_check

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "lampi_amd", "csrc")
ASM = os.path.join(CSRC, "obj", "frag_csum-gfx950.s")
HIPCC = "/opt/rocm/bin/hipcc"


def _product_asm():
    src = os.path.join(CSRC, "frag_csum.hip")
    if not os.path.exists(ASM) or os.path.getmtime(ASM) < os.path.getmtime(src):
        subprocess.run(["make", "-C", CSRC, ASM], check=True, capture_output=True)
    return open(ASM).read()


def test_product_rings_touch_no_register_in_flight():
    asm = _product_asm()
    assert isa_check.asm_loads(asm) >= 300  # the guard saw the rings (438 asm loads at r02)
    bad = isa_check.violations(asm)
    assert not bad, "\n".join(f"{k[:70]} line {ln}: {load} -> {ins}" for k, ln, load, ins in bad[:20])


def test_every_ring_kernel_names_its_waits():
    for name, (insns, _) in isa_check.parse(_product_asm()).items():
        loads = [i for i in insns if i.in_asm and isa_check._VMEM_LOAD.match(i.mn)]
        if loads:
            assert any(i.wait_regs for i in insns), name


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_guard_flags_the_round1_failure_shapes(tmp_path):
    src = os.path.join(ROOT, "tools", "isa_guard", "broken_ring.hip")
    out = tmp_path / "broken.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "--cuda-device-only", "-S", "-O3", "-std=c++17", src, "-o",
                    str(out)], check=True, capture_output=True)
    bad = isa_check.violations(out.read_text())
    kernels = {k for k, *_ in bad}
    assert any("copy_before_wait" in k for k in kernels), bad
    assert any("two_branch_waits" in k for k in kernels), bad
    assert any("refill_skipped" in k for k in kernels), bad  # round 4's ring drain
