#!/usr/bin/env python3
"""Per-kernel sums (averaged per launch) of every counter in rocprofv3 --pmc CSVs."""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
launches = collections.defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        launches[k].add((path, r["Dispatch_Id"]))
for k, v in sorted(agg.items(), key=lambda kv: -(kv[1].get("SQ_WAVE_CYCLES", 0) or kv[1].get("SQ_LDS_IDX_ACTIVE", 0))):
    n = max(1, len(launches[k]) // max(1, len(sys.argv) - 1))
    print("%-28s launches=%d %s" % (k[:28], n, {c: int(x / n) for c, x in sorted(v.items())}))
