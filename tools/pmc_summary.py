#!/usr/bin/env python3
"""Summarise tools/pmc_pass.sh output into per-kernel HBM bytes per launch.

rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB per dispatch. Corrections follow
MI355X_MICROARCH.md "HBM [CDNA4]": on gfx950 FETCH_SIZE counts exactly half the bytes of
a wide coalesced (16 B/lane) streaming read, so fetch bytes are doubled; WRITE_SIZE is
exact for 16 B/lane stores. Usage: pmc_summary.py FETCH_DIR WRITE_DIR OUT_JSON
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"]
            if not name.startswith(("dcn::", "void dcn::", "Cijk", "void ")):
                continue
            short = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            acc[short].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    fdir, wdir, out = sys.argv[1:4]
    fetch, n = per_kernel(fdir + "/run_counter_collection.csv", "FETCH_SIZE")
    write, _ = per_kernel(wdir + "/run_counter_collection.csv", "WRITE_SIZE")
    res = {}
    for k in sorted(fetch, key=lambda k: -fetch[k]):
        if not (k.startswith("dcn::") or k.startswith("Cijk")):
            continue
        fb = 2.0 * fetch[k]
        wb = write.get(k, 0.0)
        res[k] = {"launches": n[k], "fetch_bytes_raw": fetch[k], "fetch_bytes": fb,
                  "write_bytes": wb, "hbm_bytes": fb + wb}
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes, "
                     "--kernel-trace) of `bench.py --steps 2 --warmup 1`",
           "correction": "fetch_bytes = 2 x FETCH_SIZE (gfx950, MI355X_MICROARCH.md HBM section); "
                         "write_bytes = WRITE_SIZE",
           "kernels": res}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    for k, v in res.items():
        print(f"{k[:60]:60s} n={v['launches']:3d} fetch={v['fetch_bytes']/1e6:9.1f} MB "
              f"write={v['write_bytes']/1e6:9.1f} MB")


if __name__ == "__main__":
    main()
