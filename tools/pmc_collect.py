#!/usr/bin/env python3
"""profiles/<tag>_pmc_<config>.json from the PMC passes of tools/r04_pmc.sh:
for each config, the workload description and the chunk bytes (the K1
scan's algorithmic bytes, which FETCH_SIZE is calibrated on) come from the
bench line the FETCH_SIZE pass printed; tools/pmc_traffic.py does the rest.
Usage: pmc_collect.py <gpurun_out dir> <tag> [configs...]"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import pmc_traffic  # noqa: E402


def main(out_dir, tag, configs):
    root = os.path.dirname(HERE)
    for cfg in configs:
        line = os.path.join(out_dir, "pmc_fetch_%s.json" % cfg)
        fetch = os.path.join(out_dir, "pmc", "fetch_%s_counter_collection.csv" % cfg)
        write = os.path.join(out_dir, "pmc", "write_%s_counter_collection.csv" % cfg)
        if not (os.path.exists(line) and os.path.exists(fetch) and os.path.exists(write)):
            print(cfg, "missing PMC outputs")
            continue
        d = json.loads(open(line).read().strip().splitlines()[-1])
        workload = d["workload"] if "workload" in d else d["config"]["workload"]
        bytes_in = d["roofline"]["stage_alg_bytes"]["scan"]
        pmc_traffic.main(fetch, write, os.path.join(root, "profiles", "%s_pmc_%s.json" % (tag, cfg)), workload,
                         bytes_in)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:] or ["c2", "c1", "c3", "c4", "c5"])
