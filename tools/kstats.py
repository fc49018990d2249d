#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel_stats.csv into a markdown table.
usage: kstats.py <kernel_stats.csv> [title] [steps] > out.md"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
title = sys.argv[2] if len(sys.argv) > 2 else sys.argv[1]
steps = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("# %s" % title)
print()
print("total kernel time %.2f ms over the profiled run (%.2f ms per step over %g steps)" % (tot / 1e6, tot / 1e6 / steps, steps))
print()
print("| kernel | calls | total ms | % | avg us |")
print("|---|---|---|---|---|")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
    name = re.sub(r"ttdk::\(anonymous namespace\)::", "", r["Name"])
    name = re.sub(r"\(.*", "", name)[:110]
    t = float(r["TotalDurationNs"])
    print("| `%s` | %s | %.2f | %.1f | %.1f |" % (name, r["Calls"], t / 1e6, 100 * t / tot, t / 1e3 / max(1, int(r["Calls"]))))
