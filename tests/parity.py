"""GPU-vs-oracle comparison helpers (used by the -m gpu tests and smoke())."""
import numpy as np

from oracle import pyoracle as O
import pqgpu
from pqgpu import abi


def oracle_chunk(pf, rg, col):
    job, _ = pf.host_job(rg, col)
    return O.decode_chunk(job)


def compare_chunk(exp, got, where=""):
    """exp: OracleChunk; got: pqgpu.DecodedColumn.  Bit-exact comparison."""
    assert got.status == exp.status, "%s status gpu=%s oracle=%s (pages %s vs %s)" % (
        where, abi.status_name(got.status), abi.status_name(exp.status), got.error_page, exp.error_page)
    if exp.status != 0:
        assert got.error_page == exp.error_page, "%s error page %d vs %d" % (where, got.error_page, exp.error_page)
        return
    assert got.num_slots == exp.num_slots, where
    assert got.num_values == exp.num_values, where
    if exp.def_levels is not None:
        assert np.array_equal(got.def_levels, exp.def_levels), where + " def levels"
    if exp.rep_levels is not None:
        assert np.array_equal(got.rep_levels, exp.rep_levels), where + " rep levels"
    if exp.value_width == 0:
        # variable length: chars and int64 offsets[num_values + 1]
        assert got.offsets is not None and exp.offsets is not None, where + " offsets missing"
        assert np.array_equal(got.offsets, exp.offsets), where + " offsets"
        assert got.values is not None and exp.values is not None
        assert got.values.nbytes == exp.values.nbytes, "%s chars %d vs %d" % (where, got.values.nbytes,
                                                                           exp.values.nbytes)
        assert np.array_equal(got.values, exp.values), where + " chars"
    if exp.values is not None and exp.value_width > 0:
        assert got.values is not None
        assert got.values.nbytes == exp.values.nbytes, "%s values bytes %d vs %d" % (
            where, got.values.nbytes, exp.values.nbytes)
        if not np.array_equal(got.values, exp.values):
            bad = np.nonzero(got.values != exp.values)[0]
            raise AssertionError("%s values differ at %d bytes, first at byte %d" % (where, len(bad), bad[0]))
    if got.pages is not None:
        assert len(got.pages) == len(exp.pages), where
        for a, b in zip(got.pages, exp.pages):
            assert (a.page_type, a.num_values, a.not_null) == (b.page_type, b.num_values, b.not_null), where


def compare_file(data, dec, rgs=None, cols=None):
    pf = pqgpu.ParquetFile(data)
    dev = dec.upload(pf.data)
    try:
        rgs = range(pf.num_row_groups) if rgs is None else rgs
        cols = range(pf.num_columns) if cols is None else cols
        jobs, keys = [], []
        for rg in rgs:
            for c in cols:
                jobs.append(pqgpu.device_job(pf, rg, c, dev))
                keys.append((rg, c))
        res = dec.decode_jobs(jobs)
        for i, ((rg, c), r) in enumerate(zip(keys, res)):
            got = dec.download(r, i)
            exp = oracle_chunk(pf, rg, c)
            compare_chunk(exp, got, "rg%d col%d" % (rg, c))
        return res
    finally:
        dec.free(dev)


def compare_chunk_bytes(chunk, dec, **kw):
    """Hand-built chunk bytes (see pqtest_util.chunk_job) through both paths."""
    import pqtest_util as U
    keep = []
    job, buf = U.chunk_job(chunk, keep=keep, **kw)
    exp = O.decode_chunk(job)
    dev = dec.upload(buf)
    try:
        job.data = dev
        r = dec.decode_jobs([job])[0]
        got = dec.download(r, 0)
        compare_chunk(exp, got, "chunk")
        return exp, got
    finally:
        dec.free(dev)
