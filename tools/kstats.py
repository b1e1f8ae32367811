#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv as a short table (avg µs per kernel)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    n = r["Name"].split("(")[0].replace("void ", "")[:58]
    print(f"{n:58s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:9.1f} "
          f"share={float(r['TotalDurationNs'])/tot*100:5.1f}%")
