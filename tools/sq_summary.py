#!/usr/bin/env python3
"""Per-kernel sums of SQ counters from a rocprofv3 --pmc counter_collection.csv
(tools/gpu_steps.sh pmc steps), as a markdown table, with the wave-cycle
split the MI355X guide gives: WAIT_ANY (parked on s_waitcnt / barrier) +
WAIT_INST_ANY (issue stall) + ACTIVE_INST_ANY ~= WAVE_CYCLES.
Usage: sq_summary.py <counter_collection.csv> [kernel substrings...]"""
import csv
import sys
from collections import defaultdict


def main(path, picks):
    acc = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if picks and not any(p in k for p in picks):
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[k].add(r["Dispatch_Id"])
    names = sorted({c for v in acc.values() for c in v})
    print("| kernel | dispatches | " + " | ".join(names) + " | wait / issue-stall / active (of WAVE_CYCLES) |")
    print("|---|---|" + "---|" * len(names) + "---|")
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wc = v.get("SQ_WAVE_CYCLES", 0)
        split = ("%.2f / %.2f / %.2f" % (v.get("SQ_WAIT_ANY", 0) / wc, v.get("SQ_WAIT_INST_ANY", 0) / wc,
                                        v.get("SQ_ACTIVE_INST_ANY", 0) / wc)) if wc else "-"
        print("| %s | %d | " % (k[:60], len(calls[k])) + " | ".join("%.3g" % v.get(c, 0) for c in names) + " | " + split + " |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
