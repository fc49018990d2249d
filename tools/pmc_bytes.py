#!/usr/bin/env python3
"""Per-kernel HBM traffic of the last profiled training step from two rocprofv3 --pmc runs
(FETCH_SIZE, WRITE_SIZE; KB per dispatch). The step = dispatches from the last stem kernel on.
With a kernel-trace run of the same command (third argument), each kernel's time in that step
and its achieved bandwidth (bytes / time) against a 6 TB/s line.
usage: pmc_bytes.py <fetch_dir> <write_dir> [<trace_dir>]

Calibration (gfx950, rocprofv3 derived counters): FETCH_SIZE reports HALF the bytes a streaming
read moves — a 205.5 MB device copy (hipMemcpy kernel, __amd_rocclr_copyBuffer) and the BN
apply pass over a 205.5 MB tensor both read back ~100 MB, the fp32 -> bf16 cast of a 411 MB
tensor 201 MB, while WRITE_SIZE matches the bytes written (201 MB for the copy, 213 MB for the
apply with its ReLU bit mask) — profiles/r6_pmc_bytes_calibration.txt. The reads here are
therefore FETCH_SIZE x FETCH_SCALE (2)."""
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


FETCH_SCALE = 2.0
fe = [(d, n, v * FETCH_SCALE) for d, n, v in load(sys.argv[1], "FETCH_SIZE")]
wr = load(sys.argv[2], "WRITE_SIZE")
tot = defaultdict(lambda: [0.0, 0.0, 0])
for _, n, v in fe:
    tot[short(n)][0] += v
    tot[short(n)][2] += 1
for _, n, v in wr:
    tot[short(n)][1] += v
F = sum(v[0] for v in tot.values()) / 1e6
W = sum(v[1] for v in tot.values()) / 1e6
tus = defaultdict(float)
if len(sys.argv) > 3:
    f = glob.glob(sys.argv[3] + "/**/*kernel_trace.csv", recursive=True)
    rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "stem_fwd" in r["Kernel_Name"]]
    for r in rows[idx[-1]:] if idx else rows:
        tus[short(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
T = sum(tus.values())
print("step HBM traffic (reads = FETCH_SIZE x %g, calibrated): fetch" % FETCH_SCALE + " %.1f GB, write %.1f GB, total %.1f GB (%d dispatches)%s"
      % (F, W, F + W, len(fe), ", kernel time %.1f ms -> %.2f TB/s average" % (T / 1e3, (F + W) / T * 1e3) if T else ""))
print("%-100s %5s %9s %9s %9s %7s %s" % ("kernel", "n", "fetch GB", "write GB", "time us", "TB/s", "vs 6 TB/s"))
for k, v in sorted(tot.items(), key=lambda kv: -(kv[1][0] + kv[1][1]))[:60]:
    t = tus.get(k, 0.0)
    bw = (v[0] + v[1]) / t * 1e-3 if t > 0 else 0.0
    bar = ("#" * int(round(bw / 6.0 * 20))).ljust(20)[:30] if t > 0 else ""
    print("%-100s %5d %9.2f %9.2f %9.1f %7.2f |%s|" % (k, v[2], v[0] / 1e6, v[1] / 1e6, t, bw, bar))
