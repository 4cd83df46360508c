#!/usr/bin/env python3
"""Per-launch HBM traffic of each kernel from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE, separate runs: tools/gpu_pmc.sh) → JSON read by
bench.py for roofline.traffic.  Both counters are in KiB.  FETCH_SIZE is taken
raw: the gfx950 ×2 correction of MI355X_MICROARCH.md is calibrated for 16-B/lane
streaming reads only, and these kernels read with narrower, gathered loads."""
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(fetch_csv, write_csv, out, workload):
    f, w = per_kernel(fetch_csv, "FETCH_SIZE"), per_kernel(write_csv, "WRITE_SIZE")
    res = {"workload": workload, "unit": "bytes per launch", "fetch_correction": "raw (uncalibrated width)",
           "kernels": {k: {"fetch": round(f.get(k, 0.0)), "write": round(w.get(k, 0.0)),
                           "traffic": round(f.get(k, 0.0) + w.get(k, 0.0))} for k in sorted(set(f) | set(w))}}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
