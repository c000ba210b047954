"""Print facts about one kernel's gfx950 assembly (lampi_amd/csrc/obj/frag_csum-gfx950.s): scratch
traffic, lane spills, loops and the s_waitcnt vmcnt values inside them.  Usage: isa_kernel.py SUBSTRING"""
import re
import sys

S = open(sys.argv[2] if len(sys.argv) > 2 else "lampi_amd/csrc/obj/frag_csum-gfx950.s").read()
pat = sys.argv[1]
starts = [m for m in re.finditer(r"^(_Z\S+):", S, re.M) if pat in m.group(1)]
for m in starts:
    a = m.end()
    b = S.find(".Lfunc_end", a)
    body = S[a:b].split("\n")
    labels = {l.strip().split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\S+:", l)}
    scr = [i for i, l in enumerate(body) if "scratch_" in l]
    wl = sum("v_writelane" in l for l in body)
    rl = sum("v_readlane" in l for l in body)
    back = []
    for i, l in enumerate(body):
        mm = re.match(r"\s+s_(c?branch\S*)\s+(\.LBB\S+)", l)
        if mm and labels.get(mm.group(2), 1 << 30) < i:
            back.append((labels[mm.group(2)], i))
    print(m.group(1)[:140])
    print(f"  {len(body)} lines, scratch ops {len(scr)} at {scr[:20]}, writelane {wl}, readlane {rl}")
    for lo, hi in back:
        waits = [body[j].strip() for j in range(lo, hi + 1) if "vmcnt" in body[j]]
        sc = [j for j in scr if lo <= j <= hi]
        print(f"  loop {lo}-{hi}: {hi - lo} lines, scratch ops inside {len(sc)}, vmcnt waits {waits[:12]}")
