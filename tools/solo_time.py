#!/usr/bin/env python3
"""Where the last training step in a rocprofv3 kernel trace runs ALONE: the step's wall time is
split into intervals by the number of HIP streams with a kernel in flight; time with only the
main stream busy is charged to the main-stream kernel running then (those kernels have the
whole chip and set the step's critical path directly), and the step's head/tail kernels are
listed in order. A step starts at the last dispatch whose name contains --start.
usage: solo_time.py <run_kernel_trace.csv> [--start NAME] [--top N]"""
import csv
import sys
from collections import defaultdict

from trace_step import short


def main():
    path = sys.argv[1]
    start = sys.argv[sys.argv.index("--start") + 1] if "--start" in sys.argv else "stem_fwd"
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 25
    rows = list(csv.DictReader(open(path)))
    idx = [i for i, r in enumerate(rows) if start in r["Kernel_Name"]]
    last = rows[idx[-1]:] if idx else rows
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], short(r["Kernel_Name"])) for r in last]
    busy = defaultdict(float)
    for s, e, sid, _ in ks:
        busy[sid] += e - s
    main_sid = max(busy, key=busy.get)
    t0, t1 = min(k[0] for k in ks), max(k[1] for k in ks)
    ev = sorted({t0, t1} | {k[0] for k in ks} | {k[1] for k in ks})
    solo = defaultdict(float)
    none = 0.0
    multi = 0.0
    j = 0
    ks_sorted = sorted(ks)
    active = []
    for a, b in zip(ev, ev[1:]):
        while j < len(ks_sorted) and ks_sorted[j][0] <= a:
            active.append(ks_sorted[j])
            j += 1
        active = [k for k in active if k[1] > a]
        cur = [k for k in active if k[0] <= a < k[1]]
        sids = {k[2] for k in cur}
        if not cur:
            none += b - a
        elif sids == {main_sid}:
            for k in cur:
                solo[k[3]] += (b - a) / len(cur)
        else:
            multi += b - a
    wall = (t1 - t0) / 1e3
    st = sum(solo.values()) / 1e3
    print("step wall %.1f us: main stream alone %.1f us, streams overlapping %.1f us, gaps %.1f us"
          % (wall, st, multi / 1e3, none / 1e3))
    for k, v in sorted(solo.items(), key=lambda kv: -kv[1])[:top]:
        print("%9.1f us alone  %s" % (v / 1e3, k))
    print("\nfirst / last kernels of the step (start offset us, duration us, stream):")
    for k in ks_sorted[:12]:
        print("  +%9.1f %8.1f  s%s %s" % ((k[0] - t0) / 1e3, (k[1] - k[0]) / 1e3, k[2], k[3]))
    print("  ...")
    for k in ks_sorted[-12:]:
        print("  +%9.1f %8.1f  s%s %s" % ((k[0] - t0) / 1e3, (k[1] - k[0]) / 1e3, k[2], k[3]))


if __name__ == "__main__":
    main()
