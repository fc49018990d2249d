#!/usr/bin/env python3
"""Per-kernel HBM traffic of the last profiled training step from two rocprofv3 --pmc runs
(FETCH_SIZE, WRITE_SIZE; KB per dispatch). The step = dispatches from the last stem kernel on.
usage: pmc_bytes.py <fetch_dir> <write_dir>"""
import csv
import glob
import re
import sys
from collections import defaultdict


def load(d, counter):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    out = []
    for r in rows:
        if r.get("Counter_Name") != counter:
            continue
        out.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    out.sort()
    idx = [i for i, (_, n, _) in enumerate(out) if "stem_fwd" in n or "pad_channels" in n]
    return out[idx[-1]:] if idx else out


def short(n):
    n = re.sub(r"ttdk::\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n)
    return n.split("(")[0][:100]


fe = load(sys.argv[1], "FETCH_SIZE")
wr = load(sys.argv[2], "WRITE_SIZE")
tot = defaultdict(lambda: [0.0, 0.0, 0])
for _, n, v in fe:
    tot[short(n)][0] += v
    tot[short(n)][2] += 1
for _, n, v in wr:
    tot[short(n)][1] += v
F = sum(v[0] for v in tot.values()) / 1e6
W = sum(v[1] for v in tot.values()) / 1e6
print("step HBM traffic: fetch %.1f GB, write %.1f GB, total %.1f GB (%d dispatches)" % (F, W, F + W, len(fe)))
print("%-100s %5s %9s %9s" % ("kernel", "n", "fetch GB", "write GB"))
for k, v in sorted(tot.items(), key=lambda kv: -(kv[1][0] + kv[1][1]))[:45]:
    print("%-100s %5d %9.2f %9.2f" % (k, v[2], v[0] / 1e6, v[1] / 1e6))
