"""Print ms_per_step and the per-kernel HIP-event times of one bench.py JSON line."""
import json
import sys


def find(d, key):
    if isinstance(d, dict):
        if key in d:
            return d[key]
        for v in d.values():
            r = find(v, key)
            if r is not None:
                return r
    return None


d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2] if len(sys.argv) > 2 else "", d["ms_per_step"], find(d, "kernel_ms"))
