#!/usr/bin/env python3
"""Per-chunk K1 diagnostics of one bench workload: for every chunk job of the
step, pqg_debug_job's (scan path, candidates, pages, scratch, launches), plus
the stage timings of a few decodes.  scan path: 0 speculative chain, 1 serial
walk (k_scan_pages fallback), 2 prewalked (a few big pages).

    python tools/probe_jobs.py --only c2_run_heavy [--rows N]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "parquet-go_amd")]

import bench  # noqa: E402


def main():
    import argparse
    import ctypes as C
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="c2_run_heavy")
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--bits", default="1,2,4,8,12,16,20")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    args = bench.argparse.Namespace(rows=a.rows, bits=a.bits, c1_rows=10_000_000, c3_rows=200_000_000,
                                    c3gz_rows=50_000_000, c4_rows=50_000_000, c5_rows_per_rg=15_625_000)
    import pqgpu
    from pqgpu import abi
    dec = pqgpu.GpuDecoder(0)
    wl = bench.gen_workload(a.only, args, 0, 1)
    jobs = []
    for pf, specs, _ in wl.files:
        fj, dev, _ = pqgpu.span_jobs(pf, specs, dec)
        wl.devs.append(dev)
        jobs += fj
    n = len(jobs)
    arr = (abi.ChunkJob * n)(*jobs)
    res = (abi.ChunkResult * n)()
    for rep in range(a.reps):
        rc = dec.L.pqg_decode_chunks(dec.ctx, arr, n, res)
        assert rc == 0, rc
        t = dec.timings()
        print("rep %d stages(ms): %s" % (rep, " ".join("%s=%.3f" % (s, x) for s, x in zip(bench.STAGES, t[1:]))))
    for i in range(n):
        print("job %d status %d debug %s" % (i, res[i].status, dec.debug_job(i)))
    dec.close()


if __name__ == "__main__":
    main()
