#!/usr/bin/env python3
"""Per-launch HBM traffic of each kernel from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE, separate runs: tools/gpu_steps.sh pmc steps) → JSON read by
bench.py for roofline.traffic.  Both counters are in KiB.

FETCH_SIZE is calibrated on this run's own known-byte kernel: k_page_cands
reads every chunk byte exactly once with 16-byte-per-lane loads, so
factor = bytes_in / FETCH_SIZE(k_page_cands) (MI355X_MICROARCH.md: gfx950
reports 1/2 of such streaming reads, factor ~2).  `fetch` applies that factor
to every kernel; `fetch_raw` keeps the counter as read.  tools/fetch_calib.hip
(profiles/r04/fetch_calib) checks the other widths the kernels use: 4-byte
coalesced loads report the same 1/2; 4-byte random gathers from a 256 KiB or
a 4 MiB table report only the table's compulsory misses (8 XCDs x table / 2):
gathers served by L2 never reach the counter, so a gather kernel's fetch above
its streams is lines re-fetched from the Infinity Cache after eviction.
WRITE_SIZE is exact for 16-byte streaming stores and taken as is."""
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


def main(fetch_csv, write_csv, out, workload, bytes_in):
    f, w = per_kernel(fetch_csv, "FETCH_SIZE"), per_kernel(write_csv, "WRITE_SIZE")
    cal = f.get("pqg::k_page_cands", 0.0)
    factor = float(bytes_in) / cal if cal > 0 else 1.0
    res = {"workload": workload, "unit": "bytes per launch",
           "fetch_correction": {"factor": round(factor, 4),
                                "calibrated_on": "k_page_cands: every chunk byte read once, 16 B per lane "
                                                 "(bytes_in = %d)" % int(bytes_in)},
           "kernels": {k: {"fetch_raw": round(f.get(k, 0.0)), "fetch": round(f.get(k, 0.0) * factor),
                           "write": round(w.get(k, 0.0)),
                           "traffic": round(f.get(k, 0.0) * factor + w.get(k, 0.0))}
                       for k in sorted(set(f) | set(w))}}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}))


if __name__ == "__main__":
    main(*sys.argv[1:6])
