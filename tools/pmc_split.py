"""Summarise an SQ PMC pass (rocprofv3 --pmc ... -o run --output-format csv) per kernel:
counters per dispatch and as a fraction of SQ_WAVE_CYCLES. Usage: pmc_split.py DIR [substr]"""
import collections
import csv
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "gemm_split"
rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"]
    if sub not in k:
        continue
    short = k[k.find(sub):][:80]
    agg[short][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(short, r["Counter_Name"])] += 1
for k, v in agg.items():
    n = max(cnt[(k, c)] for c in v)
    wc = v.get("SQ_WAVE_CYCLES", 0) or 1
    print(k, f"({n} dispatches)")
    for c in sorted(v):
        print(f"   {c:28s} {v[c] / n:16.0f}  {v[c] / wc:.3f}")
