#!/usr/bin/env python3
"""Turn rocprofv3 PMC CSVs of a bench.py run into per-launch HBM traffic (profiles/traffic.json).

Recipe (/opt/skills/guides/MI355X_MICROARCH.md, HBM section): FETCH_SIZE is collected in its
own pass (no trace domains); on gfx950 it reports exactly half of the bytes of a wide
coalesced streaming read, so read bytes = 2 x FETCH_SIZE x 1024.  TCC_EA0_RDREQ (64-B units)
is reported beside it as a cross-check.  Values are per dispatch of the named kernel,
averaged over the profiled launches.

WRITE_SIZE (its own pass, --write) reads the bytes exactly for 16-B-per-lane streaming stores
(same guide section); with it, hbm_bytes_per_launch = read + written bytes (fused copies).
--skip/--take select matched dispatches in dispatch order (a bench run that launches one kernel
template for several layouts in turn).

Usage: tools/pmc_traffic.py --fetch gpurun_out/pmc_fetch --ea gpurun_out/pmc_ea \
           --kernel crc_regular_kernel --key crc_4194304x4096 --out profiles/traffic.json
"""
import argparse
import collections
import csv
import glob
import json
import os


def per_dispatch(root, kernel_substr, skip=0, take=None, last=None):
    files = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)
    if os.path.isfile(root):
        files = [root]
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in files:
        for r in csv.DictReader(open(f)):
            if kernel_substr not in r["Kernel_Name"]:
                continue
            vals[(f, int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
    out = [vals[k] for k in sorted(vals)][skip:]
    if last:
        out = out[-last:]
    return out if take is None else out[:take]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--ea")
    ap.add_argument("--write", help="WRITE_SIZE pass (fused copies: traffic = read + written bytes)")
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--take", type=int, default=None)
    ap.add_argument("--last", type=int, default=None, help="only the last N matching dispatches (after warm-ups)")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--key", required=True)
    ap.add_argument("--algorithmic-bytes", type=int, required=True)
    ap.add_argument("--out", default="profiles/traffic.json")
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    fd = per_dispatch(a.fetch, a.kernel, a.skip, a.take, a.last)
    if not fd:
        raise SystemExit(f"no dispatches of {a.kernel} in {a.fetch}")
    fetch_kb = sum(d["FETCH_SIZE"] for d in fd) / len(fd)
    entry = {
        "kernel": a.kernel,
        "dispatches": len(fd),
        "FETCH_SIZE_kB": fetch_kb,
        "hbm_bytes_per_launch": int(2 * fetch_kb * 1024),  # gfx950: FETCH_SIZE = 1/2 of wide reads
        "algorithmic_bytes_per_launch": a.algorithmic_bytes,
        "correction": "x2 (gfx950 FETCH_SIZE counts 128-B requests at 64 B, MI355X_MICROARCH.md HBM section)",
        "source": a.source,
    }
    if a.write:
        wd = per_dispatch(a.write, a.kernel, a.skip, a.take, a.last)
        if not wd:
            raise SystemExit(f"no dispatches of {a.kernel} in {a.write}")
        write_kb = sum(d["WRITE_SIZE"] for d in wd) / len(wd)
        entry["WRITE_SIZE_kB"] = write_kb
        entry["read_bytes_per_launch"] = entry["hbm_bytes_per_launch"]
        entry["write_bytes_per_launch"] = int(write_kb * 1024)
        entry["hbm_bytes_per_launch"] += int(write_kb * 1024)
        entry["correction"] += "; WRITE_SIZE x1 (exact for 16-B-per-lane streaming stores)"
    if a.ea:
        ed = per_dispatch(a.ea, a.kernel)
        if ed:
            rd = sum(d.get("TCC_EA0_RDREQ_sum", 0.0) for d in ed) / len(ed)
            rd32 = sum(d.get("TCC_EA0_RDREQ_32B_sum", 0.0) for d in ed) / len(ed)
            entry["TCC_EA0_RDREQ_sum"] = rd
            entry["TCC_EA0_RDREQ_32B_sum"] = rd32
            entry["ea_bytes_64B_units"] = int(rd * 64)
    entry["traffic_over_algorithmic"] = entry["hbm_bytes_per_launch"] / a.algorithmic_bytes
    d = {}
    if os.path.exists(a.out):
        d = json.load(open(a.out))
    d[a.key] = entry
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(d, open(a.out, "w"), indent=1)
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
