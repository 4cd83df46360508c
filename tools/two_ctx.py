#!/usr/bin/env python3
"""Experiment: the C2 batch split over K decode contexts (K HIP streams), each
decoding its share of the chunks asynchronously, against one context decoding
all of them.  Prints ms per step for K = 1 and K.

    python tools/two_ctx.py [--only c2] [--k 2] [--steps 10]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "parquet-go_amd")]

import bench  # noqa: E402


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="c2")
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    args = bench.argparse.Namespace(rows=100_000_000, bits="1,2,4,8,12,16,20", c1_rows=10_000_000,
                                    c3_rows=200_000_000, c3gz_rows=50_000_000, c4_rows=50_000_000,
                                    c5_rows_per_rg=15_625_000)
    import pqgpu
    from pqgpu import abi
    decs = [pqgpu.GpuDecoder(0) for _ in range(a.k)]
    wl = bench.gen_workload(a.only, args, 0, 1)
    jobs = []
    for pf, specs, _ in wl.files:
        fj, dev, _ = pqgpu.span_jobs(pf, specs, decs[0])
        wl.devs.append(dev)
        jobs += fj
    n = len(jobs)
    L = decs[0].L
    # K = 1
    arr = (abi.ChunkJob * n)(*jobs)
    res = (abi.ChunkResult * n)()
    for d in decs:
        L.pqg_set_timing(d.ctx, 0)
    for _ in range(3):
        assert L.pqg_decode_chunks(decs[0].ctx, arr, n, res) == 0
    t0 = time.perf_counter()
    for _ in range(a.steps):
        assert L.pqg_decode_chunks(decs[0].ctx, arr, n, res) == 0
    t1 = time.perf_counter()
    print("k=1: %.4f ms/step" % ((t1 - t0) / a.steps * 1e3))
    # K contexts: chunks dealt round-robin
    parts = [[j for i, j in enumerate(jobs) if i % a.k == k] for k in range(a.k)]
    arrs = [(abi.ChunkJob * len(p))(*p) for p in parts]
    ress = [(abi.ChunkResult * len(p))() for p in parts]

    def step():
        for d, ar, p in zip(decs, arrs, parts):
            assert L.pqg_decode_chunks_async(d.ctx, ar, len(p)) == 0
        for d, r, p in zip(decs, ress, parts):
            assert L.pqg_sync(d.ctx, r, len(p)) == 0

    for _ in range(3):
        step()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    t1 = time.perf_counter()
    print("k=%d: %.4f ms/step" % (a.k, (t1 - t0) / a.steps * 1e3))
    for r, p in zip(ress, parts):
        assert all(r[i].status == 0 for i in range(len(p)))
    for d in decs:
        d.close()


if __name__ == "__main__":
    main()
