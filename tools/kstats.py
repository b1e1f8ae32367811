#!/usr/bin/env python3
"""Print rocprofv3 kernel stats (µs) of one or more profile dirs, filtered by substring.
Usage: kstats.py DIR [DIR ...] [--match=a,b] [--top=N]"""
import csv
import glob
import sys

dirs = [a for a in sys.argv[1:] if not a.startswith("--")]
match = None
top = None
for a in sys.argv[1:]:
    if a.startswith("--match="):
        match = a.split("=", 1)[1].split(",")
    if a.startswith("--top="):
        top = int(a.split("=", 1)[1])
for d in dirs:
    f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)
    if not f:
        print(d, "(no stats)")
        continue
    print(d)
    for i, r in enumerate(csv.DictReader(open(f[0]))):
        if top is not None and i >= top:
            break
        n = r["Name"]
        if match and not any(m in n for m in match):
            continue
        print(f"  {int(r['Calls']):4d} {float(r['AverageNs']) / 1e3:9.1f} us  {n[:90]}")
