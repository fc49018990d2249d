#!/usr/bin/env python3
"""Per-kernel breakdown of the LAST training step in a rocprofv3 kernel trace (a step starts
at the last dispatch whose name contains --start, default pad_channels). Prints total kernel
time, step wall time and the top kernels, plus the ordered list of BN streaming passes with
their durations (for per-layer bandwidth checks).
--streams adds a per-HIP-stream table (busy time and top kernels of each stream).
usage: trace_step.py <run_kernel_trace.csv> [--start NAME] [--seq SUBSTR] [--streams]"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"ttdk::\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"\(.*$", "", n) if not n.startswith("big::") else n.split("(")[0]
    return n[:110]


def main():
    path = sys.argv[1]
    start = sys.argv[sys.argv.index("--start") + 1] if "--start" in sys.argv else "pad_channels"
    seqf = sys.argv[sys.argv.index("--seq") + 1] if "--seq" in sys.argv else None
    rows = list(csv.DictReader(open(path)))
    idx = [i for i, r in enumerate(rows) if start in r["Kernel_Name"]]
    last = rows[idx[-1]:] if idx else rows
    tot, cnt = defaultdict(float), defaultdict(int)
    for r in last:
        n = short(r["Kernel_Name"])
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[n] += t
        cnt[n] += 1
        if seqf and seqf in n:
            print("%9.1f us  grid=%s %s" % (t, r["Grid_Size_X"], n))
    s = sum(tot.values())
    wall = (int(last[-1]["End_Timestamp"]) - int(last[0]["Start_Timestamp"])) / 1e3
    print("step: kernel %.1f us, wall %.1f us, %d dispatches" % (s, wall, len(last)))
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:30]:
        print("%9.1f us %5.1f%% n=%4d %s" % (v, 100 * v / s, cnt[k], k))
    if "--streams" in sys.argv:
        per = defaultdict(lambda: defaultdict(float))
        for r in last:
            per[r["Stream_Id"]][short(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        for sid, d in sorted(per.items()):
            busy = sum(d.values())
            print("\nstream %s: busy %.1f us (%.1f%% of wall)" % (sid, busy, 100 * busy / wall))
            for k, v in sorted(d.items(), key=lambda kv: -kv[1])[:25]:
                print("%9.1f us %5.1f%% %s" % (v, 100 * v / busy, k))


if __name__ == "__main__":
    main()
