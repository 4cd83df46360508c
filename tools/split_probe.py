#!/usr/bin/env python3
"""Probe: the C2 chunks split over K contexts (K HIP streams on one GPU),
launched async and synced together, against one context.  Prints ms/step."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "parquet-go_amd")]
import pqgpu  # noqa: E402
from pqgpu import abi  # noqa: E402
from gen import pqwrite as W  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
ks = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,2,3").split(",")]
files = [f[1] for f in W.config_c2_family(rows=rows)]
base = pqgpu.GpuDecoder(0)
jobs = []
for data in files:
    pf = pqgpu.ParquetFile(data)
    dev = base.upload(pf.data)
    jobs.append(pqgpu.device_job(pf, 0, 0, dev))
order = [6, 0, 5, 1, 4, 2, 3]  # heavy widths first, dealt round robin
for K in ks:
    decs = [base] + [pqgpu.GpuDecoder(0) for _ in range(K - 1)]
    parts = [[jobs[order[i]] for i in range(len(order)) if i % K == k] for k in range(K)]
    arrs = [(abi.ChunkJob * len(p))(*p) for p in parts]
    ress = [(abi.ChunkResult * len(p))() for p in parts]

    def step():
        for d, a, p in zip(decs, arrs, parts):
            assert d.L.pqg_decode_chunks_async(d.ctx, a, len(p)) == 0
        for d, r, p in zip(decs, ress, parts):
            assert d.L.pqg_sync(d.ctx, r, len(p)) == 0
    for _ in range(3):
        step()
    assert all(r[i].status == 0 for r, p in zip(ress, parts) for i in range(len(p)))
    t = time.perf_counter()
    for _ in range(20):
        step()
    ms = (time.perf_counter() - t) / 20 * 1e3
    print("K=%d %.3f ms/step" % (K, ms), flush=True)
    for d in decs[1:]:
        d.close()
