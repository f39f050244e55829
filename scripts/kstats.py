#!/usr/bin/env python3
"""Median per-kernel duration from a rocprofv3 kernel_trace.csv (robust to one-off setup launches).
usage: kstats.py <dir with run_kernel_trace.csv>"""
import collections
import csv
import sys

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1].rstrip("/") + "/run_kernel_trace.csv")):
    d[r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
rows = sorted(((sorted(v)[len(v) // 2], k, len(v)) for k, v in d.items()), reverse=True)
for med, k, n in rows:
    print(f"{k[:60]:60s} {n:6d}  median {med:9.2f} us")
