#!/usr/bin/env python3
"""Print bench.py JSON lines (one per run, as the A/B scripts append them) as a table: workload, mode, roofline
fraction, kernel ms, parity.  Usage: tools/ab/jsonl_table.py FILE.jsonl [LABEL ...] -- LABELs (one per line, in
order) replace the workload text."""
import json
import sys

rows = [json.loads(x) for x in open(sys.argv[1]) if x.strip().startswith("{")]
labels = sys.argv[2:]
for i, d in enumerate(rows):
    r = d.get("roofline", {})
    w = labels[i] if i < len(labels) else str(d.get("config", {}).get("workload", ""))[:60]
    p = d.get("parity", {}).get("ok")
    print(f"{w:60s} {d.get('dtype', '')} frac {r.get('frac')} kernel_ms {r.get('kernel_avg_ms')} parity {p}")
