#!/usr/bin/env python3
"""Per-kernel PMC summary of one profiled run (rocprofv3 --pmc ... --kernel-trace): for every
kernel name with at least --min dispatches, counters averaged per dispatch plus derived ratios
(MFMA busy %, wait / active % of wave cycles, HBM TB/s from FETCH_SIZE + WRITE_SIZE over the
traced duration). Several run directories (one counter pass each) are merged by kernel name.
usage: pmc_kernels.py <dir> [<dir> ...] [--min N] [--top K]"""
import csv
import glob
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"ttdk::\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n)
    return n.split("(")[0][:90]


def main():
    dirs = [a for i, a in enumerate(sys.argv[1:], 1) if not a.startswith("--") and sys.argv[i - 1] not in ("--min", "--top")]
    mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 3
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 20
    ctr = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values per dispatch
    dur = defaultdict(list)
    files = [f for d in dirs for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True)]
    for f in files:
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
        for (disp, c), v in per.items():
            ctr[names[disp]][c].append(v)
    for f in [f for d in dirs[:1] for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True)]:
        for r in csv.DictReader(open(f)):
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = []
    for k, cs in ctr.items():
        n = max(len(v) for v in cs.values())
        if n < mn:
            continue
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        us = sum(dur[k]) / len(dur[k]) if dur.get(k) else 0.0
        rows.append((us * n, k, n, us, avg))
    rows.sort(reverse=True)
    for tot, k, n, us, v in rows[:top]:
        out = ["%-90s n=%4d  %8.1f us" % (k, n, us)]
        if v.get("GRBM_GUI_ACTIVE") and v.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
            cyc = v["GRBM_GUI_ACTIVE"] / 8
            out.append("MFMA busy %5.1f%%" % (100 * v["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024)))
        if v.get("SQ_WAVE_CYCLES"):
            wc = v["SQ_WAVE_CYCLES"]
            out.append("wait_any %4.1f%% wait_inst %4.1f%% active %4.1f%%" % (
                100 * v.get("SQ_WAIT_ANY", 0) / wc, 100 * v.get("SQ_WAIT_INST_ANY", 0) / wc,
                100 * v.get("SQ_ACTIVE_INST_ANY", 0) / wc))
        if v.get("SQ_INSTS_MFMA"):
            out.append("VALU/MFMA %.2f" % (v.get("SQ_INSTS_VALU", 0) / v["SQ_INSTS_MFMA"]))
        if "FETCH_SIZE" in v and us > 0:
            gb = (v["FETCH_SIZE"] + v.get("WRITE_SIZE", 0)) / 1e6  # KB -> GB
            out.append("HBM %.2f GB %.2f TB/s" % (gb, gb / us * 1e3))
        if v.get("SQ_LDS_IDX_ACTIVE"):
            out.append("LDS conflict %.1f%%" % (100 * v.get("SQ_LDS_BANK_CONFLICT", 0) / v["SQ_LDS_IDX_ACTIVE"]))
        print("  ".join(out))


if __name__ == "__main__":
    main()
