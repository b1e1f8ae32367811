#!/usr/bin/env python3
"""Per-kernel average of every counter in rocprofv3 counter_collection.csv files.
Usage: pmc_table.py DIR [DIR ...] [--match dcn::]"""
import csv
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = "dcn::"
for a in sys.argv[1:]:
    if a.startswith("--match="):
        match = a.split("=", 1)[1]
acc = defaultdict(lambda: defaultdict(list))
for d in args:
    with open(d + "/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            if match in k:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.1f}")
