#!/usr/bin/env python3
"""Count kernel dispatches per name in a rocprofv3 kernel trace CSV.
usage: launch_count.py TRACE.csv [NAME_SUBSTR]"""
import csv
import sys
from collections import Counter

c = Counter()
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if len(sys.argv) < 3 or sys.argv[2] in n:
        c[n[:110]] += 1
for n, k in c.most_common():
    print("%5d  %s" % (k, n))
