#!/usr/bin/env python3
"""Round 6: per-launch HBM traffic from the PMC passes of tools/ab/r6_pmc.sh (profiles/r06/pmc/), written into
profiles/traffic.json.  Read bytes = 2 x FETCH_SIZE x 1024 (gfx950 counts a 128-byte request at 64 B), written
bytes = WRITE_SIZE x 1024 (MI355X_MICROARCH.md HBM section); every value is the mean over the last launches of
one bench phase (a phase = consecutive dispatches of one kernel; bench.py's census launches every 16th call split
a phase into blocks of 16, which are joined back by the phase boundaries below)."""
import collections
import csv
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PMC = os.path.join(ROOT, "profiles", "r06", "pmc")


def dispatches(tag, counter, kernel, fname=None):
    """(dispatch id, value) of every dispatch of `kernel` (substring) in the pass, in order."""
    path = os.path.join(PMC, f"{tag}_{fname or counter}.csv")
    per = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]:
            d = int(r["Dispatch_Id"])
            per[d] = per.get(d, 0.0) + float(r["Counter_Value"])
    return sorted(per.items())


def mean(v):
    return sum(v) / len(v)


def phase(tag, counter, kernel, lo, hi=None, nth=0, size=None, last=5, fname=None):
    """Mean of the last `last` dispatches of the nth run of consecutive dispatches whose value lies in [lo, hi)
    (runs of `size` dispatches when given: bench phases of warm-up + timed calls)."""
    vals = [v for _, v in dispatches(tag, counter, kernel, fname) if v >= lo and (hi is None or v < hi)]
    if size:
        vals = vals[nth * size:(nth + 1) * size]
    return mean(vals[-last:]), len(vals)


def entry(kernel, fetch_kb, write_kb, alg, src, extra=None):
    rd = 2.0 * fetch_kb * 1024
    e = {"kernel": kernel, "FETCH_SIZE_kB": f"{fetch_kb:.1f}", "read_bytes_per_launch": str(int(rd)),
         "correction": "x2 (gfx950 FETCH_SIZE counts 128-B requests at 64 B, MI355X_MICROARCH.md HBM section)",
         "algorithmic_bytes_per_launch": str(alg), "source": src}
    tot = rd
    if write_kb is not None:
        wr = write_kb * 1024
        e["WRITE_SIZE_kB"] = f"{write_kb:.1f}"
        e["write_bytes_per_launch"] = str(int(wr))
        e["correction"] += "; WRITE_SIZE x 1024 (exact for 16-byte stores)"
        tot += wr
    e["hbm_bytes_per_launch"] = str(int(tot))
    e["traffic_over_algorithmic"] = f"{tot / alg:.5f}"
    if extra:
        e.update(extra)
    return e


def main():
    path = os.path.join(ROOT, "profiles", "traffic.json")
    t = json.load(open(path))
    B = 4194304 * 4096
    GM = 16384 * 65456
    src = "profiles/r06/pmc/{}_{{FETCH,WRITE}}_SIZE.csv (round 6, tools/ab/r6_pmc.sh: bench.py {}; {})"
    # fused copies, CRC: lampi_msg_bcopy (crc_light_copy_kernel), then the descriptor batches (crc_light_frag_copy
    # <CopySource>: aligned, src + 8, dst + 8, dst + 1, 105 calls each), then GM's send slots (crc_light_copy_kernel)
    f, _ = phase("bcopy_crc", "FETCH_SIZE", "crc_light_copy_kernel", 4e6)
    w, _ = phase("bcopy_crc", "WRITE_SIZE", "crc_light_copy_kernel", 8e6)
    t["crc_bcopy_4194304x4096"] = entry("crc_light_copy_kernel", f, w, 2 * B,
                                        src.format("bcopy_crc", "--bcopy", "lampi_msg_bcopy 4M x 4 KiB"))
    for nth, key, what in [(0, "crc_bcopy_desc_4194304x4096", "descriptors, aligned"),
                           (1, "crc_bcopy_desc_src8", "descriptors, n-1 sources at + 8")]:
        f, _ = phase("bcopy_crc", "FETCH_SIZE", "crc_light_frag_copy_kernel", 4e6, size=105, nth=nth)
        w, _ = phase("bcopy_crc", "WRITE_SIZE", "crc_light_frag_copy_kernel", 8e6, size=105, nth=nth)
        t[key] = entry("crc_light_frag_copy_kernel<CopySource>", f, w, 2 * B if nth == 0 else 2 * (B - 4096),
                       src.format("bcopy_crc", "--bcopy", what))
    f, _ = phase("bcopy_crc", "FETCH_SIZE", "crc_light_copy_kernel", 1e5, 4e6)
    w, _ = phase("bcopy_crc", "WRITE_SIZE", "crc_light_copy_kernel", 2e5, 8e6)
    t["crc_bcopy_gm_slots"] = entry("crc_light_copy_kernel", f, w, 2 * GM,
                                    src.format("bcopy_crc", "--bcopy", "gm_send_slots: 16,384 x 65,456 B into "
                                               "64 KiB slots after the 72-byte header"))
    # SUM: lampi_msg_bcopy (sum_copy_row_kernel), descriptors (sum_copy_wg_kernel), GM slots (sum_copy_row_kernel)
    f, _ = phase("bcopy_sum", "FETCH_SIZE", "sum_copy_row_kernel", 4e6)
    w, _ = phase("bcopy_sum", "WRITE_SIZE", "sum_copy_row_kernel", 8e6)
    t["sum_bcopy_4194304x4096"] = entry("sum_copy_row_kernel", f, w, 2 * B,
                                        src.format("bcopy_sum", "--bcopy --mode sum", "lampi_msg_bcopy 4M x 4 KiB"))
    f, _ = phase("bcopy_sum", "FETCH_SIZE", "sum_copy_wg_kernel", 4e6, size=105, nth=0)
    w, _ = phase("bcopy_sum", "WRITE_SIZE", "sum_copy_wg_kernel", 8e6, size=105, nth=0)
    t["sum_bcopy_desc_4194304x4096"] = entry("sum_copy_wg_kernel<CopySource>", f, w, 2 * B,
                                             src.format("bcopy_sum", "--bcopy --mode sum", "descriptors, aligned"))
    f, _ = phase("bcopy_sum", "FETCH_SIZE", "sum_copy_row_kernel", 1e5, 4e6)
    w, _ = phase("bcopy_sum", "WRITE_SIZE", "sum_copy_row_kernel", 2e5, 8e6)
    t["sum_bcopy_gm_slots"] = entry("sum_copy_row_kernel", f, w, 2 * GM,
                                    src.format("bcopy_sum", "--bcopy --mode sum", "gm_send_slots"))
    # packed rows (round 6): config A's shape and 64-byte fragments (the results' writes counted for 64 B)
    f, _ = phase("packedA_crc", "FETCH_SIZE", "crc_regular_kernel", 1e5)
    t["crc_1048576x1024"] = entry("crc_regular_kernel<kSub = 16> (packed rows)", f, None, 1048576 * 1024,
                                  "profiles/r06/pmc/packedA_crc_FETCH_SIZE.csv (round 6: bench.py --frags 1048576 "
                                  "--frag-bytes 1024 --seed 1)")
    f, _ = phase("packed64_crc", "FETCH_SIZE", "crc_regular_kernel", 1e5)
    w, _ = phase("packed64_crc", "WRITE_SIZE", "crc_regular_kernel", 1e4)
    t["crc_16777216x64"] = entry("crc_regular_kernel<kSub = 1> (packed rows)", f, w, 16777216 * 64,
                                 "profiles/r06/pmc/packed64_crc_{FETCH,WRITE}_SIZE.csv (round 6: bench.py --frags "
                                 "16777216 --frag-bytes 64; writes = the 4-byte results, 6.25% of the payload)")
    # config C: FETCH_SIZE and the SQ instruction counts per 4 KiB row of payload
    f, _ = phase("configC", "FETCH_SIZE", "crc_stream_kernel", 1e6)
    rows = 4295007488 / 4096
    valu, _ = phase("configC", "SQ_INSTS_VALU", "crc_stream_kernel", 1)
    lds, _ = phase("configC", "SQ_INSTS_LDS", "crc_stream_kernel", 1, fname="SQ_INSTS_VALU")
    t["crc_configC"] = entry("crc_stream_kernel", f, None, 4295007488,
                             "profiles/r06/pmc/configC_FETCH_SIZE.csv (round 6: bench.py --config C)",
                             {"sq_per_4KiB_row": {"SQ_INSTS_VALU": round(valu / rows, 1), "SQ_INSTS_LDS": round(lds / rows, 1),
                                                  "source": "profiles/r06/pmc/configC_SQ_INSTS_VALU.csv (round 6, own "
                                                            "pass: SQ_INSTS_VALU, SQ_INSTS_LDS, SQ_WAVES)"}})
    # config B on the round-6 final library (tools/ab/r6_pmc_b.sh), when its passes are present
    if os.path.exists(os.path.join(PMC, "B6_FETCH_SIZE.csv")):
        f, _ = phase("B6", "FETCH_SIZE", "crc_regular_kernel", 1e6)
        w, _ = phase("B6", "WRITE_SIZE", "crc_regular_kernel", 1)
        rowsB = B / 4096
        sq = {c: round(phase("B6", c, "crc_regular_kernel", 1, fname="SQ_INSTS_VALU")[0] / rowsB, 1)
              for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU")}
        sq["source"] = "profiles/r06/pmc/B6_SQ_INSTS_VALU.csv (round 6 final library, own pass)"
        t["crc_4194304x4096"] = entry("crc_regular_kernel", f, w, B,
                                      "profiles/r06/pmc/B6_{FETCH,WRITE}_SIZE.csv (round 6 final library, "
                                      "tools/ab/r6_pmc_b.sh: bench.py; writes = the 4-byte results)",
                                      {"sq_per_4KiB_row": sq})
        f, _ = phase("desc6", "FETCH_SIZE", "crc_regular_kernel", 1e6)
        t["crc_desc_4194304x4096"] = entry("crc_regular_kernel<kDesc>", f, None, B,
                                           "profiles/r06/pmc/desc6_FETCH_SIZE.csv (round 6 final library: bench.py "
                                           "--desc; reads include the 64 MiB of descriptors)")
    json.dump(t, open(path, "w"), indent=1)
    for k in ["crc_4194304x4096", "crc_desc_4194304x4096", "crc_bcopy_4194304x4096", "crc_bcopy_desc_4194304x4096", "crc_bcopy_desc_src8", "crc_bcopy_gm_slots",
              "sum_bcopy_4194304x4096", "sum_bcopy_desc_4194304x4096", "sum_bcopy_gm_slots", "crc_1048576x1024",
              "crc_16777216x64", "crc_configC"]:
        print(k, t[k]["traffic_over_algorithmic"], t[k].get("sq_per_4KiB_row", ""))


if __name__ == "__main__":
    main()
