#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection.csv files: per kernel (name filter), average
of each counter over dispatches, plus derived ratios.
usage: pmc_summary.py <dir with p*/run_counter_collection.csv> [kernel-substring]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else "gemm"
vals = defaultdict(list)
name = None
for f in sorted(glob.glob(d + "/p*/run_counter_collection.csv")):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if filt not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"][:100]
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    agg = defaultdict(list)
    for (disp, c), v in per.items():
        agg[c].append(v)
    for c, l in agg.items():
        vals[c] = sum(l) / len(l)
print(name)
for c in sorted(vals):
    print("  %-28s %16.0f" % (c, vals[c]))
v = vals
if v.get("SQ_WAVE_CYCLES"):
    wc = v["SQ_WAVE_CYCLES"]
    print("  wait_any %.1f%%  wait_inst %.1f%%  active %.1f%%  (of wave cycles)" % (
        100 * v.get("SQ_WAIT_ANY", 0) / wc, 100 * v.get("SQ_WAIT_INST_ANY", 0) / wc,
        100 * v.get("SQ_ACTIVE_INST_ANY", 0) / wc))
if v.get("GRBM_GUI_ACTIVE") and v.get("SQ_VALU_MFMA_BUSY_CYCLES"):
    # MFMA busy cycles are summed over SIMDs (256 CUs x 4); GUI_ACTIVE is GPU cycles
    print("  MFMA util %.1f%%" % (100 * v["SQ_VALU_MFMA_BUSY_CYCLES"] / (v["GRBM_GUI_ACTIVE"] * 1024)))
if v.get("SQ_LDS_IDX_ACTIVE"):
    print("  LDS bank-conflict cycles %.1f%% of LDS active" % (100 * v.get("SQ_LDS_BANK_CONFLICT", 0) / v["SQ_LDS_IDX_ACTIVE"]))
