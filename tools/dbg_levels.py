#!/usr/bin/env python3
"""Diagnostic: decode the page-by-page C2 case and print where the GPU's def levels differ from the oracle's."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "parquet-go_amd"), os.path.join(ROOT, "tests")]
import pqgpu  # noqa: E402
from pqgpu import abi  # noqa: E402
from gen import pqwrite as W  # noqa: E402
from oracle import pyoracle as O  # noqa: E402
import pqtest_util as U  # noqa: E402
import test_boundary as TB  # noqa: E402

dec = pqgpu.GpuDecoder(0)
data = W.config_c2(rows=9000, bits=7, rows_per_page=2500)[0]
pf = pqgpu.ParquetFile(data)
m = pf.chunk_meta(0, 0)
chunk = pf.data[m.start:m.start + m.total_compressed_size]
desc = pf.columns[0].desc
dsc = abi.ColumnDesc()
C.memmove(C.byref(dsc), C.byref(desc), C.sizeof(dsc))
dsc.codec = m.codec
kw = dict(max_def=desc.max_def, max_rep=desc.max_rep, codec=m.codec, type_length=desc.type_length)
dict_page, pages = TB._page_parts(chunk, desc.physical_type, **kw)
for i, page in enumerate(pages):
    exp_job, _ = U.chunk_job(dict_page + page, ptype=desc.physical_type, **kw)
    exp = O.decode_chunk(exp_job)
    got = TB._decode_page(dec, dsc, page, dict_page)
    a, b = np.asarray(got.def_levels), np.asarray(exp.def_levels)
    bad = np.nonzero(a != b)[0] if a.shape == b.shape else None
    print("page", i, "slots", len(b), "status", got.status, exp.status, "mismatch",
          None if bad is None else (len(bad), bad[:20].tolist()))
    if bad is not None and len(bad):
        j = bad[0]
        print("  got", a[max(0, j - 8):j + 24].tolist())
        print("  exp", b[max(0, j - 8):j + 24].tolist())
# whole chunk too
job = pqgpu.device_job(pf, 0, 0, dec.upload(pf.data))
r = dec.decode_jobs([job])[0]
got = dec.download(r, 0)
exp = O.decode_chunk(pf.host_job(0, 0)[0])
a, b = np.asarray(got.def_levels), np.asarray(exp.def_levels)
bad = np.nonzero(a != b)[0]
print("chunk mismatch", len(bad), bad[:20].tolist())
