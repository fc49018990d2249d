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
    # MFMA busy cycles are summed over SIMDs (256 CUs x 4); GRBM_GUI_ACTIVE is summed over the
    # 8 XCDs' GRBMs (each counts the dispatch's GPU cycles): cycles = GUI_ACTIVE / 8. Checked
    # against wall time: 65536x4096x1024 bf16 -> 8.78M / 8 = 1.10M cycles = 457 us at 2.4 GHz
    # = 1.20 PFLOP/s, and MFMA busy / (cycles x 1024) = 47.8 % of the 2.5 PFLOP/s dense peak.
    cyc = v["GRBM_GUI_ACTIVE"] / 8
    print("  kernel %.0f cycles (%.1f us at 2.4 GHz)" % (cyc, cyc / 2400))
    print("  MFMA util %.1f%%" % (100 * v["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024)))
if v.get("TCC_EA0_RDREQ_sum") is not None and v.get("TCC_EA0_WRREQ_sum") is not None:
    print("  HBM requests (EA0) rd %.0f wr %.0f" % (v["TCC_EA0_RDREQ_sum"], v["TCC_EA0_WRREQ_sum"]))
if v.get("SQ_LDS_IDX_ACTIVE"):
    print("  LDS bank-conflict cycles %.1f%% of LDS active" % (100 * v.get("SQ_LDS_BANK_CONFLICT", 0) / v["SQ_LDS_IDX_ACTIVE"]))
