#!/usr/bin/env python3
"""One step of a rocprofv3 kernel trace as a timeline (start, end, duration in us, queue).

Usage: tools/timeline.py RUN_kernel_trace.csv STEP_KERNEL_SUBSTRING [--gaps]
A step is the span between two launches of the kernel whose name contains
STEP_KERNEL_SUBSTRING; the shortest such span is printed (the eager timed steps, not the
profiled passes with their timing events). --gaps adds the idle time on the step kernel's
queue between consecutive kernels, and its total.
"""
import csv
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    gaps = "--gaps" in sys.argv
    rows = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
    idx = [i for i, x in enumerate(rows) if key in x["Kernel_Name"]]
    if len(idx) < 2:
        sys.exit(f"fewer than two launches of {key!r} in {path}")
    best = min(zip(idx, idx[1:]),
               key=lambda ab: int(rows[ab[1]]["Start_Timestamp"]) - int(rows[ab[0]]["Start_Timestamp"]))
    a, b = best
    t0 = int(rows[a]["Start_Timestamp"])
    q0 = rows[a]["Queue_Id"]
    step = (int(rows[b]["Start_Timestamp"]) - t0) / 1000
    print(f"# step {step:.1f} us ({path}, steps delimited by {key!r})")
    print(f"# {'start':>8} {'end':>8} {'dur':>7} {'queue':>5} {'gap':>6}  kernel")
    prev_end, idle = None, 0.0
    for x in rows[a:b]:
        s = (int(x["Start_Timestamp"]) - t0) / 1000
        e = (int(x["End_Timestamp"]) - t0) / 1000
        gap = ""
        if gaps and x["Queue_Id"] == q0:
            if prev_end is not None and s > prev_end:
                idle += s - prev_end
                gap = f"{s - prev_end:6.1f}"
            prev_end = max(prev_end or 0.0, e)
        print(f"  {s:8.1f} {e:8.1f} {e - s:7.1f} {'q' + x['Queue_Id']:>5} {gap:>6}  {x['Kernel_Name'][:70]}")
    if gaps:
        tail = step - (prev_end or 0.0)
        print(f"# idle on queue {q0}: {idle:.1f} us between kernels + {tail:.1f} us to the next step")


if __name__ == "__main__":
    main()
