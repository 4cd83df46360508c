#!/usr/bin/env python3
"""profiles/<tag>_pmc_<config>.json from the PMC passes of tools/gpu_steps.sh
(steps pmc:<cfg>:FETCH_SIZE and pmc:<cfg>:WRITE_SIZE): for each config, the
workload description and the chunk bytes (the K1 scan's algorithmic bytes,
which FETCH_SIZE is calibrated on) come from the bench line the FETCH_SIZE
pass printed; tools/pmc_traffic.py does the rest.
Usage: pmc_collect.py <gpurun_out/TAG dir> <tag> [configs...]"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import pmc_traffic  # noqa: E402


def main(out_dir, tag, configs):
    root = os.path.dirname(HERE)
    for cfg in configs:
        line = os.path.join(out_dir, "pmc_%s_FETCH_SIZE.out" % cfg)
        fetch = os.path.join(out_dir, "pmc", "%s_FETCH_SIZE_counter_collection.csv" % cfg)
        write = os.path.join(out_dir, "pmc", "%s_WRITE_SIZE_counter_collection.csv" % cfg)
        if not (os.path.exists(line) and os.path.exists(fetch) and os.path.exists(write)):
            print(cfg, "missing PMC outputs")
            continue
        d = json.loads(open(line).read().strip().splitlines()[-1])
        workload = d["workload"] if "workload" in d else d["config"]["workload"]
        bytes_in = d["roofline"]["stage_alg_bytes"]["scan"]
        out = os.path.join(root, "profiles", "%s_pmc_%s.json" % (tag, cfg))
        pmc_traffic.main(fetch, write, out, workload, bytes_in)
        res = json.load(open(out))
        if not 1.8 <= res["fetch_correction"]["factor"] <= 2.2:
            # k_page_cands no longer reads every chunk byte when the K1 prewalk
            # takes a chunk (C5's one-page chunks): the calibrated gfx950 factor
            # of the other configs (1.99) instead
            raw = sum(v["fetch_raw"] for k, v in res["kernels"].items() if k.startswith("pqg::k_page_cands"))
            pmc_traffic.main(fetch, write, out, workload, 1.99 * raw)
            res = json.load(open(out))
            res["fetch_correction"]["calibrated_on"] = ("the other configs' k_page_cands factor (1.99): here the K1 "
                                                        "prewalk takes some chunks, so k_page_cands reads fewer than "
                                                        "bytes_in = %d" % int(bytes_in))
            json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:] or ["c2", "c1", "c3", "c4", "c5"])
