#!/usr/bin/env python3
"""Diagnostic: test_levels' random def streams (maxd 2), where the GPU's def levels differ from the oracle's."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "parquet-go_amd"), os.path.join(ROOT, "tests")]
import pqgpu  # noqa: E402
from pqgpu import abi  # noqa: E402
from oracle import pyoracle as O  # noqa: E402
import pqtest_util as U  # noqa: E402
import test_levels as TL  # noqa: E402

dec = pqgpu.GpuDecoder(0)
maxd = 2
rng = np.random.default_rng(maxd)
for it in range(3):
    data = TL.chunk(rng, 12, maxd, 0)
    job, buf = U.chunk_job(data, ptype=abi.INT32, max_def=maxd)
    exp = O.decode_chunk(job)
    dev = dec.upload(np.frombuffer(data, dtype=np.uint8))
    job.data = dev
    r = dec.decode_jobs([job])[0]
    got = dec.download(r, 0)
    print("status", got.status, exp.status, "slots", got.num_slots, exp.num_slots, "nn", got.num_values, exp.num_values)
    a, b = np.asarray(got.def_levels), np.asarray(exp.def_levels)
    bad = np.nonzero(a != b)[0]
    starts = np.cumsum([0] + [p.num_values for p in exp.pages if p.page_type in (0, 3)])
    print("page starts", starts.tolist())
    print("mismatch", len(bad), bad[:40].tolist())
    for j in bad[:5]:
        print(j, "got", a[max(0, j - 4):j + 12].tolist(), "exp", b[max(0, j - 4):j + 12].tolist())
