"""Static guard for the asm-issued load rings in gfx950 device assembly (test infrastructure).

The hot kernels issue their HBM loads with inline asm and wait for them with explicit
`s_waitcnt vmcnt(N)` asm statements that take the destination registers as in/out operands
(4.5 "Waits chosen at run time").  The compiler cannot see those loads: nothing
but the machine code itself keeps an instruction from reading, copying or overwriting a load's
destination registers before the data has landed.  Round 1 hit this twice (a spilled in-flight
register; a phi copy of in-flight ring registers before the asm wait -- one wrong checksum in
3,000).  This module checks the invariant on the compiler's final assembly of every kernel:

    from every asm-issued vector-memory load, on every control-flow path, the first
    instruction that touches any of its destination VGPRs must be the asm wait that names
    them (every wait statement lists its operands in a `; lampi-wait <regs>` comment) or a
    full `s_waitcnt vmcnt(0)`; anything else -- a copy, a read, an overwrite, a store of the
    registers -- is a violation.

Input: the `.s` of frag_csum.hip built with the library's own flags (lampi_amd/csrc/Makefile,
obj/frag_csum-gfx950.s); inline asm appears between `;;#ASMSTART` / `;;#ASMEND` with its
operands substituted, numeric local labels (`1f`, `3b`) included.

Usage: violations(asm_text) -> [(kernel, line_no, load_line, offending_line)]
"""
from __future__ import annotations

import re

_FUNC = re.compile(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$")
_LABEL = re.compile(r"^(\.L\w+|\d+):\s*(;.*)?$")
_VREG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
_VMEM_LOAD = re.compile(r"^(global|buffer|flat|scratch)_load_\w+$")
_END = ("s_endpgm", "s_setpc_b64", "s_trap")


def _vregs(text: str) -> set[int]:
    out = set()
    for m in _VREG.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


class Insn:
    __slots__ = ("line", "text", "mn", "ops", "in_asm", "wait_regs", "target", "regs")

    def __init__(self, line, text, mn, ops, in_asm, wait_regs, target):
        self.line, self.text, self.mn, self.ops = line, text, mn, ops
        self.in_asm, self.wait_regs, self.target = in_asm, wait_regs, target
        self.regs = _vregs(ops)


def parse(asm: str):
    """{kernel: (insns, labels)}; labels: name -> [insn index] (numeric labels may repeat)."""
    funcs = {}
    name, insns, labels, in_asm = None, None, None, False
    for no, raw in enumerate(asm.splitlines(), 1):
        line = raw.strip()
        if not line:
            continue
        m = _FUNC.match(line)
        if m and not line.startswith(".") and not line[0].isdigit():
            name, insns, labels, in_asm = m.group(1), [], {}, False
            funcs[name] = (insns, labels)
            continue
        if name is None:
            continue
        if line.startswith(".Lfunc_end"):
            name = None
            continue
        if line.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if line.startswith(";;#ASMEND"):
            in_asm = False
            continue
        m = _LABEL.match(line)
        if m:
            labels.setdefault(m.group(1), []).append(len(insns))
            continue
        code, _, comment = line.partition(";")
        code = code.strip()
        wait = _vregs(comment) if "lampi-wait" in comment else None
        if not code:
            if wait is not None:  # a comment-only wait marker (after the run-time selected waits)
                insns.append(Insn(no, line, "", "", in_asm, wait, None))
            continue
        if code.startswith("."):
            continue  # directives
        mn, _, ops = code.partition(" ")
        target = None
        if mn == "s_branch" or mn.startswith("s_cbranch"):
            target = ops.strip()
        insns.append(Insn(no, line, mn, ops.strip(), in_asm, wait, target))
    return funcs


def _resolve(labels, target, i):
    """Index of the branch target from insn i (numeric local labels: Nf next, Nb previous)."""
    m = re.fullmatch(r"(\d+)([fb])", target)
    if m:
        pos = labels.get(m.group(1), [])
        if m.group(2) == "f":
            nxt = [p for p in pos if p > i]
            return min(nxt) if nxt else None
        prv = [p for p in pos if p <= i]
        return max(prv) if prv else None
    pos = labels.get(target)
    return pos[0] if pos else None


def _succ(insns, labels, i):
    ins = insns[i]
    if ins.mn in _END:
        return []
    out = []
    if ins.target is not None:
        t = _resolve(labels, ins.target, i)
        if t is not None:
            out.append(t)
        if ins.mn == "s_branch":
            return out
    if i + 1 < len(insns):
        out.append(i + 1)
    return out


def check_kernel(insns, labels):
    """[(load insn, offending insn)] for every asm load whose registers are touched before their wait."""
    bad = []
    for li, load in enumerate(insns):
        if not (load.in_asm and _VMEM_LOAD.match(load.mn)) or " lds" in f" {load.ops} ":
            continue
        dest = _vregs(load.ops.split(",")[0])
        seen, stack = set(), list(_succ(insns, labels, li))
        while stack:
            j = stack.pop()
            if j in seen:
                continue
            seen.add(j)
            ins = insns[j]
            if ins.wait_regs is not None and dest & ins.wait_regs:
                if not dest <= ins.wait_regs:
                    bad.append((load, ins))  # a wait covering only part of the load
                continue  # this path waits for the load by name
            if ins.mn == "s_waitcnt" and re.search(r"vmcnt\(0\)", ins.ops):
                continue  # everything retired
            if ins.regs & dest:
                bad.append((load, ins))
                continue
            stack.extend(_succ(insns, labels, j))
    return bad


def violations(asm: str):
    res = []
    for name, (insns, labels) in parse(asm).items():
        for load, ins in check_kernel(insns, labels):
            res.append((name, ins.line, load.text, ins.text))
    return res


def asm_loads(asm: str) -> int:
    """Number of asm-issued vector-memory loads (so a test can assert the guard saw the rings)."""
    n = 0
    for insns, _ in parse(asm).values():
        n += sum(1 for i in insns if i.in_asm and _VMEM_LOAD.match(i.mn))
    return n
