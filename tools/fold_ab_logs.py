"""Fold raw same-box A/B sweep logs (one tiny log per variant x round) into one markdown table per
sweep directory, so the numbers stay in the tree without hundreds of two-line files.
python tools/fold_ab_logs.py OUT.md DIR [DIR ...]   (each DIR under profiles/)"""
import json
import os
import re
import sys


def numbers(path):
    """The measured fractions of a log: bench.py JSON lines (every 'frac' it holds) or the
    microbenchmarks' 'x.xxx of 8 TB/s' / '%' lines."""
    out = []
    for line in open(path, errors="replace"):
        line = line.strip()
        if line.startswith("{"):
            try:
                d = json.loads(line)
            except ValueError:
                continue
            fr = {}
            for k, v in d.items():
                if isinstance(v, dict) and "frac" in v:
                    fr["value" if k == "roofline" else k] = round(v["frac"], 4)
            ok = d.get("parity", {}).get("ok") if isinstance(d.get("parity"), dict) else None
            out.append(", ".join(f"{k} {v}" for k, v in fr.items()) + (f", parity {ok}" if ok is not None else ""))
        elif re.search(r"of 8 TB/s|%|GiB/s|\bms\b", line) and "amdgpu.ids" not in line:
            out.append(re.sub(r"\s+", " ", line)[:160])
    return out


def main():
    dst, dirs = sys.argv[1], sys.argv[2:]
    lines = ["# Round-2 A/B sweeps, folded", "",
             "Each row is one raw log of a same-box A/B sweep (variant, bench arguments, round), with the",
             "fractions of the 8 TB/s roofline it reported.  DESIGN.md cites the conclusions; the raw",
             "two-line logs were folded here by tools/fold_ab_logs.py.", ""]
    for d in dirs:
        lines += [f"## {d}", "", "| log | measured |", "|---|---|"]
        for root, _, files in sorted(os.walk(d)):
            for f in sorted(files):
                p = os.path.join(root, f)
                for i, n in enumerate(numbers(p) or ["(no numbers)"]):
                    lines.append(f"| {os.path.relpath(p, d) if i == 0 else ''} | {n.replace('|', '/')} |")
        lines.append("")
    with open(dst, "w") as fh:
        fh.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
