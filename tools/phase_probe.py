#!/usr/bin/env python3
"""Diagnostic: run a C2 / C3 / C4 decode a few times with the -DPQG_PROFILE library and
print the in-kernel phase cycle counters (PQG_LIB=.../libpqgpu_prof.so)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "parquet-go_amd")]
import pqgpu  # noqa: E402
from gen import pqwrite as W  # noqa: E402
from pqgpu import abi  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
cfg = sys.argv[2] if len(sys.argv) > 2 else "c2"
if cfg.startswith("c2"):  # c2 (every width) or c2:b1,b2,... (those widths)
    bits = [int(b) for b in cfg[3:].split(",")] if ":" in cfg else [1, 2, 4, 8, 12, 16, 20]
    files = [f[1] for f in W.config_c2_family(rows=rows, bits_list=bits)]
elif cfg == "c3_gzip":
    files = [W.config_c3(rows=rows, codec=W.GZIP)[0]]
elif cfg == "c4":
    files = [W.config_c4(rows=rows)[0]]
else:
    files = [W.config_c3(rows=rows)[0]]
dec = pqgpu.GpuDecoder(0)
jobs = []
for data in files:
    pf = pqgpu.ParquetFile(data)
    dev = dec.upload(pf.data)
    jobs.append(pqgpu.device_job(pf, 0, 0, dev))
arr = (abi.ChunkJob * len(jobs))(*jobs)
res = (abi.ChunkResult * len(jobs))()
out = (C.c_uint64 * 192)()
for it in range(3):
    assert dec.L.pqg_decode_chunks(dec.ctx, arr, len(jobs), res) == 0
    k = dec.L.pqg_debug_counters(dec.ctx, out, 192)
    print("iter", it, "timings", ["%.3f" % x for x in dec.timings()])
    print("  counters", {i: out[i] for i in range(k) if out[i]})
