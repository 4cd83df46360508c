"""Quirk policy (DESIGN.md "Quirk policy"): Q1 and Q2 are
caller-side stitching defects of parquet-go's readPageData / readPages.  The
decoder (libpqgpu, and the oracle's pqo_decode_chunk) stitches
spec-correctly; the oracle's pqo_decode_column_store reproduces the reference's
ColumnStore.values contents for triage, on hand-built 2-row-group x 2-page
dictionary files with nulls.

Expected reference contents are derived here from the cited lines directly:
  Q1  readPageData appends each page's numValues-long slice: notNull values,
      then numValues - notNull nils (chunk_reader.go:394-397, page_v1.go:27-55).
  Q2  from row group 2 on, the dictionary page decodes into the store's reused
      backing array (chunk_reader.go:235, page_dict.go:50-53); the first data
      page's append overwrites entries [0, numValues) of it, so the second data
      page's keys below that read page 1's slots (type_dict.go:39-59)."""
import numpy as np
import pytest

import pqgpu
from gen import pqwrite as W
from oracle import pyoracle as O
from pqgpu import abi

ROWS = 4000  # 2 row groups x 2 pages of 1000 rows


def _file(seed=3, d=6):
    rng = np.random.default_rng(seed)
    defs = (rng.random(ROWS) >= 0.3).astype(np.uint8)
    dvals = (np.arange(d, dtype=np.int32) + 1) * 111
    vals = dvals[rng.integers(0, d, size=int(defs.sum()))]
    col = W.Column("q", W.INT32, vals, repetition=W.OPTIONAL, encoding=W.RLE_DICTIONARY, def_levels=defs,
                   rows_per_page=ROWS // 4)
    return W.write_file([col], ROWS, row_groups=2)


def _chunks(data):
    pf = pqgpu.ParquetFile(data)
    jobs = [pf.host_job(rg, 0)[0] for rg in range(pf.num_row_groups)]
    return pf, jobs, [O.decode_chunk(j) for j in jobs]


def _page_slices(ch):
    """(num_values, not_null, values int32) per data page of a spec decode."""
    out, vo = [], 0
    vals = ch.values.view(np.int32)
    for p in ch.pages:
        if p.page_type == abi.PAGE_DICTIONARY:
            continue
        out.append((p.num_values, p.not_null, vals[vo:vo + p.not_null]))
        vo += p.not_null
    return out


def test_product_rejects_quirk_mask():
    job = abi.ChunkJob()
    job.quirks = abi.QUIRK_Q1_PAGE_NILS
    assert job.quirks == 1  # libpqgpu returns INVALID_ARG for it (pqg_runtime.hip; needs a GPU to call)


def test_no_quirks_is_the_spec_decode():
    pf, jobs, chs = _chunks(_file())
    store = O.decode_column_store(jobs, 0)
    for (st, vals, nil), ch in zip(store, chs):
        assert st == 0 and not nil.any()
        assert np.array_equal(vals, ch.values)


def test_q1_page_nils():
    pf, jobs, chs = _chunks(_file())
    store = O.decode_column_store(jobs, abi.QUIRK_Q1_PAGE_NILS)
    for (st, vals, nil), ch in zip(store, chs):
        assert st == 0
        exp_v, exp_nil = [], []
        for n, nn, v in _page_slices(ch):
            exp_v += list(v) + [0] * (n - nn)
            exp_nil += [0] * nn + [1] * (n - nn)
        assert np.array_equal(vals.view(np.int32), np.array(exp_v, np.int32))
        assert np.array_equal(nil, np.array(exp_nil, np.uint8))
        # the defect: ColumnStore.get pops values in order, so once a page has
        # nulls the rows after it read the nils instead of later values
        assert len(exp_v) == ch.num_slots > ch.num_values


def test_q2_dictionary_alias_second_row_group():
    data = _file()
    pf, jobs, chs = _chunks(data)
    q12 = abi.QUIRK_Q1_PAGE_NILS | abi.QUIRK_Q2_DICT_ALIAS
    store = O.decode_column_store(jobs, q12)
    q1 = O.decode_column_store(jobs, abi.QUIRK_Q1_PAGE_NILS)
    # row group 1 starts from an empty store: no aliasing yet
    assert np.array_equal(store[0][1], q1[0][1]) and np.array_equal(store[0][2], q1[0][2])
    # row group 2: the dictionary decodes into row group 1's backing array;
    # page 1 is decoded intact, then its append overwrites the dictionary
    ch = chs[1]
    dict_vals = []
    for v in ch.values.view(np.int32):  # the writer numbers dictionary entries by first appearance
        if v not in dict_vals:
            dict_vals.append(int(v))
    (n1, nn1, v1), (n2, nn2, v2) = _page_slices(ch)
    page1_slots = [(int(x), 0) for x in v1] + [(0, 1)] * (n1 - nn1)
    live = [(x, 0) for x in dict_vals]
    for k in range(min(n1, len(live))):
        live[k] = page1_slots[k]
    exp2 = [live[dict_vals.index(int(x))] for x in v2] + [(0, 1)] * (n2 - nn2)
    got_v = store[1][1].view(np.int32)
    got_nil = store[1][2]
    assert [(int(a), int(b)) for a, b in zip(got_v[:n1], got_nil[:n1])] == page1_slots
    assert [(int(a), int(b)) for a, b in zip(got_v[n1:], got_nil[n1:])] == exp2
    assert not np.array_equal(got_v, q1[1][1].view(np.int32))  # the defect is visible


def test_q2_requires_q1():
    _, jobs, _ = _chunks(_file())
    arr = (abi.ChunkJob * len(jobs))(*jobs)
    out = (O.StoreRG * len(jobs))()
    assert O.lib().pqo_decode_column_store(arr, len(jobs), abi.QUIRK_Q2_DICT_ALIAS, out) == abi.STATUS_CODES["INVALID_ARG"]


@pytest.mark.parametrize("size,exp", [(1, 8), (8, 8), (9, 16), (33, 48), (1025, 1152), (32768, 32768),
                                      (32769, 40960)])
def test_go_size_classes_sample(size, exp):
    """Spot values of the Go 1.13 size-class rounding the Q2 emulation uses
    (runtime/sizeclasses.go; outside /root/reference: parity unpinned)."""
    import ctypes as C
    L = O.lib()
    if not hasattr(L, "pqo_go_roundupsize"):
        pytest.skip("not exported")
    L.pqo_go_roundupsize.restype = C.c_int64
    assert L.pqo_go_roundupsize(C.c_int64(size)) == exp


def _store_equal(a, b):
    assert a[0] == b[0] == 0
    assert np.array_equal(a[2], b[2])
    if isinstance(a[1], tuple):
        assert np.array_equal(a[1][0], b[1][0]) and np.array_equal(a[1][1], b[1][1])
    else:
        assert np.array_equal(a[1], b[1])


def _store_reads_equal(spec, quirky):
    """What ColumnStore.get pops (data_store.go:158-203: the next store entry
    for each slot with dLevel == maxD, in order) is the same: the quirky store
    starts with the spec store's entries, and Q1's page-tail nils (one page:
    only at the chunk's end) are never reached."""
    assert spec[0] == quirky[0] == 0
    n = len(spec[2])
    assert not spec[2].any()
    assert np.array_equal(quirky[2][:n], spec[2]) and quirky[2][n:].all()
    if isinstance(spec[1], tuple):
        (c0, o0), (c1, o1) = spec[1], quirky[1]
        assert np.array_equal(o1[:n + 1], o0) and np.array_equal(c1[:o0[-1]], c0)
    else:
        w = len(spec[1]) // max(n, 1)
        assert np.array_equal(quirky[1][:n * w], spec[1])


def test_c5_fixture_is_quirk_free():
    """the C5 fixture must not trigger Q1/Q2, so that page-level
    parity (GPU == oracle) is also parity with parquet-go's own NextRow.  Every
    chunk with nulls or a dictionary has exactly one data page (the layout of
    parquet-go's writer, chunk_writer.go:237-246), and the reference's
    column-store contents with Q1|Q2 reproduced equal the spec decode over
    three row groups in what ColumnStore.get reads, for every column (byte
    arrays included)."""
    rows = 50_000  # > 20 000 rows: the other columns have several pages
    data, _ = W.config_c5(row_groups=(0, 1, 2), rows_per_rg=rows)
    pf = pqgpu.ParquetFile(data)
    assert pf.num_row_groups == 3
    q12 = abi.QUIRK_Q1_PAGE_NILS | abi.QUIRK_Q2_DICT_ALIAS
    for c in range(pf.num_columns):
        jobs = [pf.host_job(rg, c)[0] for rg in range(3)]
        for j in jobs:
            ch = O.decode_chunk(j)
            assert ch.status == 0
            data_pages = [p for p in ch.pages if p.page_type != abi.PAGE_DICTIONARY]
            has_dict = any(p.page_type == abi.PAGE_DICTIONARY for p in ch.pages)
            has_nulls = ch.num_values < ch.num_slots
            if has_dict or has_nulls:
                assert len(data_pages) == 1, (pf.columns[c].path, len(data_pages))
        spec = O.decode_column_store(jobs, 0)
        quirky = O.decode_column_store(jobs, q12)
        for rg in range(3):
            _store_reads_equal(spec[rg], quirky[rg])


def test_byte_array_store_q2_alias():
    """pqo_decode_column_store on byte arrays: a 2-row-group x 2-page string
    dictionary column shows Q2 from the second row group on (the store's
    entries after page 1 differ from the spec decode), not in the first."""
    rng = np.random.default_rng(5)
    words = [b"w%02d" % i for i in range(6)]
    keys = rng.integers(0, 6, size=ROWS)
    lens = np.array([len(words[k]) for k in keys])
    offs = np.zeros(ROWS + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    chars = np.frombuffer(b"".join(words[k] for k in keys), np.uint8).copy()
    col = W.Column("s", W.BYTE_ARRAY, chars, offsets=offs, encoding=W.RLE_DICTIONARY, rows_per_page=ROWS // 4)
    data = W.write_file([col], ROWS, row_groups=2)
    pf = pqgpu.ParquetFile(data)
    jobs = [pf.host_job(rg, 0)[0] for rg in range(2)]
    spec = O.decode_column_store(jobs, 0)
    q12 = O.decode_column_store(jobs, abi.QUIRK_Q1_PAGE_NILS | abi.QUIRK_Q2_DICT_ALIAS)
    _store_equal(spec[0], q12[0])
    (c0, o0), (c1, o1) = spec[1][1], q12[1][1]
    assert len(o0) == len(o1) == ROWS // 2 + 1
    assert not (np.array_equal(c0, c1) and np.array_equal(o0, o1))
    # the spec store is the chunk's own decode
    ch = O.decode_chunk(jobs[1])
    assert np.array_equal(c0, ch.values) and np.array_equal(o0, ch.offsets)
