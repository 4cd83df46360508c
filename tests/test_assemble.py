"""K8 level assembly (validity bitmap, spaced values, record/list offsets).

The oracle (oracle/pq_oracle.cpp pqo_assemble) walks the ColumnStore.get
cursors one slot at a time (data_store.go:158-203).  It is pinned against the
reference's TwitterBlog vectors (data_store_test.go:346-389) and against the
closed-form definition; the GPU tests compare pqg_assemble with it bit for bit.
"""
import json
import os

import numpy as np
import pytest

from oracle import pyoracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _nested_offsets(rows):
    """Record offsets and inner-list offsets of TwitterBlog's [[...], [...]] rows."""
    rec, inner, n = [0], [0], 0
    for row in rows:
        for lst in row:
            n += len(lst)
            inner.append(n)
        rec.append(n)
    return rec, inner


def _closed_form(defs, reps, vals, max_def, level, w):
    n = len(defs) if defs is not None else len(reps)
    valid = np.ones(n, bool) if defs is None else (np.asarray(defs) == max_def)
    bnd = np.ones(n, bool) if reps is None else (np.asarray(reps) <= level)
    validity = np.packbits(valid, bitorder="little")
    spaced = np.zeros((n, w), np.uint8)
    if w:
        dense = np.asarray(vals).view(np.uint8).reshape(-1, w)
        spaced[valid] = dense[: int(valid.sum())]
    offsets = np.append(np.flatnonzero(bnd), n).astype(np.int64)
    return validity, spaced.reshape(-1), offsets, (int(valid.sum()), n - int(valid.sum()), int(bnd.sum()))


def _random_case(rng, n, max_def, with_rep, w):
    defs = rng.integers(0, max_def + 1, size=n).astype(np.uint8) if max_def else None
    if defs is not None:
        defs[rng.random(n) < 0.6] = max_def
    reps = rng.integers(0, 3, size=n).astype(np.uint8) if with_rep else None
    nv = n if defs is None else int((defs == max_def).sum())
    vals = rng.integers(0, 256, size=max(nv * w, 1), dtype=np.uint8)[: nv * w]
    return defs, reps, vals


def test_oracle_twitter_blog_offsets():
    g = json.load(open(os.path.join(GOLD, "dremel.json")))
    rec, inner = _nested_offsets(g["rows"])
    d, r = np.array(g["def_levels"]), np.array(g["rep_levels"])
    vals = np.array(g["values"], np.int32)
    validity, spaced, off0, cnt = O.assemble(d, r, vals, g["max_def"], 0, 4)
    assert off0.tolist() == rec and cnt == (10, 0, 2)
    assert spaced.view(np.int32).tolist() == g["values"]
    _, _, off1, _ = O.assemble(d, r, vals, g["max_def"], 1, 4)
    assert off1.tolist() == inner


@pytest.mark.parametrize("n", [0, 1, 7, 64, 4097, 20011])
@pytest.mark.parametrize("max_def,with_rep,w", [(1, False, 4), (3, True, 8), (2, True, 12), (0, True, 1)])
def test_oracle_matches_closed_form(n, max_def, with_rep, w):
    rng = np.random.default_rng(n * 31 + max_def)
    defs, reps, vals = _random_case(rng, n, max_def, with_rep, w)
    got = O.assemble(defs, reps, vals, max_def, 1, w) if defs is not None else \
        O.assemble(None, reps, vals, max_def, 1, w)
    exp = _closed_form(defs, reps, vals, max_def, 1, w)
    assert np.array_equal(got[0], exp[0]) and np.array_equal(got[1], exp[1])
    assert np.array_equal(got[2], exp[2]) and got[3] == exp[3]


# ---------------------------------------------------------------- GPU parity

@pytest.fixture(scope="module")
def dec():
    import pqgpu
    d = pqgpu.GpuDecoder(0)
    yield d
    d.close()


def _gpu_assemble(dec, defs, reps, vals, max_def, level, w):
    n = len(defs) if defs is not None else len(reps)
    dp = dec.upload(defs) if defs is not None else None
    rp = dec.upload(reps) if reps is not None else None
    vp = dec.upload(np.ascontiguousarray(vals).view(np.uint8)) if w else None
    a, vb, sb, ob = dec.assemble(dp, rp, vp, n, max_def, level, w, validity=True, spaced=w > 0, offsets=True)
    validity = dec.d2h(vb, (n + 7) // 8)
    spaced = dec.d2h(sb, n * w) if w else np.zeros(0, np.uint8)
    offsets = dec.d2h(ob, (a.num_boundaries + 1) * 8, np.int64)
    for p in (dp, rp, vp, vb, sb, ob):
        if p:
            dec.free(p)
    return validity, spaced, offsets, (a.num_valid, a.null_count, a.num_boundaries)


def _check(got, exp):
    assert np.array_equal(got[0], exp[0]), "validity"
    assert np.array_equal(got[1], exp[1]), "spaced values"
    assert np.array_equal(got[2], exp[2]), "offsets"
    assert tuple(got[3]) == tuple(exp[3]), "counts"


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 4095, 4096, 4097, 100_003, 1_000_000])
@pytest.mark.parametrize("max_def,with_rep,w,level", [(1, False, 4, 0), (3, True, 8, 0), (3, True, 8, 1),
                                                       (2, True, 12, 0), (0, True, 1, 0), (1, False, 0, 0)])
def test_gpu_assemble_random(dec, n, max_def, with_rep, w, level):
    rng = np.random.default_rng(n + 7 * max_def + w)
    defs, reps, vals = _random_case(rng, n, max_def, with_rep, w)
    if defs is None and reps is None:
        reps = np.zeros(n, np.uint8)
    exp = O.assemble(defs, reps, vals, max_def, level, w)
    _check(_gpu_assemble(dec, defs, reps, vals, max_def, level, w), exp)


@pytest.mark.gpu
def test_gpu_assemble_twitter_blog(dec):
    g = json.load(open(os.path.join(GOLD, "dremel.json")))
    rec, inner = _nested_offsets(g["rows"])
    d = np.array(g["def_levels"], np.uint8)
    r = np.array(g["rep_levels"], np.uint8)
    v = np.array(g["values"], np.int32)
    got0 = _gpu_assemble(dec, d, r, v, g["max_def"], 0, 4)
    got1 = _gpu_assemble(dec, d, r, v, g["max_def"], 1, 4)
    assert got0[2].tolist() == rec and got1[2].tolist() == inner
    assert got0[1].view(np.int32).tolist() == g["values"]


@pytest.mark.gpu
def test_gpu_assemble_decoded_chunks(dec):
    """Decode → assemble on the device result arrays, vs oracle decode → oracle
    assemble: a C2-shaped optional int32 chunk and a LIST<double> (C5 shape)."""
    import pqgpu
    import parity as P
    from gen import pqwrite as W
    rng = np.random.default_rng(5)
    rows = 30000
    rep, defs, vals = [], [], []
    for _ in range(rows):
        k = int(rng.integers(0, 4))
        if rng.random() < 0.05:
            rep.append(0); defs.append(0)
        elif k == 0:
            rep.append(0); defs.append(1)
        else:
            for j in range(k):
                rep.append(0 if j == 0 else 1)
                if rng.random() < 0.05:
                    defs.append(2)
                else:
                    defs.append(3); vals.append(rng.standard_normal())
    lst = W.Column("l", W.DOUBLE, np.array(vals), repetition=W.LIST, def_levels=np.array(defs),
                   rep_levels=np.array(rep), rows_per_page=2500)
    files = [W.write_file([lst], rows, row_groups=1), W.config_c2(rows=50_000, bits=8, rows_per_page=20000)[0]]
    for data in files:
        pf = pqgpu.ParquetFile(data)
        devp = dec.upload(pf.data)
        try:
            r = dec.decode_jobs([pqgpu.device_job(pf, 0, 0, devp)])[0]
            assert r.status == 0
            exp_chunk = P.oracle_chunk(pf, 0, 0)
            md = pf.columns[0].desc.max_def
            w = r.value_width
            exp = O.assemble(exp_chunk.def_levels, exp_chunk.rep_levels, exp_chunk.values, md, 0, w)
            a, vb, sb, ob = dec.assemble(r.def_levels, r.rep_levels, r.values, r.num_slots, md, 0, w,
                                         validity=True, spaced=True, offsets=True)
            got = (dec.d2h(vb, (r.num_slots + 7) // 8), dec.d2h(sb, r.num_slots * w),
                   dec.d2h(ob, (a.num_boundaries + 1) * 8, np.int64), (a.num_valid, a.null_count, a.num_boundaries))
            _check(got, exp)
            assert a.num_valid == r.num_values
            assert a.num_boundaries == rows if data is files[0] else True
            for p in (vb, sb, ob):
                dec.free(p)
        finally:
            dec.free(devp)


@pytest.mark.gpu
def test_gpu_assemble_multi_pass_scan(dec):
    """> 4096 segments (16 M slots): the segment scan takes several block passes."""
    rng = np.random.default_rng(77)
    n = (1 << 24) + 3 * 4096 + 17
    defs, reps, vals = _random_case(rng, n, 3, True, 4)
    exp = O.assemble(defs, reps, vals, 3, 0, 4)
    _check(_gpu_assemble(dec, defs, reps, vals, 3, 0, 4), exp)


# ---------------------------------------------------------------- K8 list export (Arrow LIST)

def _c5_list_chunk(rows=40_000, rg=0):
    import pqgpu
    import parity as P
    from gen import pqwrite as W
    data, _ = W.config_c5(row_groups=(rg,), rows_per_rg=rows)
    pf = pqgpu.ParquetFile(data)
    return data, pf, P.oracle_chunk(pf, 0, 0)


def test_oracle_list_export_matches_pyarrow():
    """pqo_assemble_list on the oracle's decode of C5's LIST<double> chunk equals
    pyarrow's ListArray (an independent reader): offsets, list validity, element
    validity and element values."""
    import io
    import pyarrow.parquet as pq
    data, pf, ch = _c5_list_chunk()
    lv, lo, ev, evals, cnt = O.assemble_list(ch.def_levels, ch.rep_levels, ch.values, 3, 1, 2, 8)
    arr = pq.read_table(io.BytesIO(data)).column("lst").combine_chunks()
    rows = len(arr)
    assert cnt[0] == rows and cnt[3] == arr.null_count
    assert np.array_equal(lo, np.asarray(arr.offsets))
    assert np.array_equal(np.unpackbits(lv, bitorder="little")[:rows].astype(bool), np.asarray(arr.is_valid()))
    flat = arr.values
    assert cnt[1] == len(flat) and cnt[2] == len(flat) - flat.null_count
    assert np.array_equal(np.unpackbits(ev, bitorder="little")[:cnt[1]].astype(bool), np.asarray(flat.is_valid()))
    got = evals.view(np.float64)
    exp = np.asarray(flat.fill_null(0.0))
    assert np.array_equal(got.view(np.uint64), exp.view(np.uint64))


def _random_lists(rng, rows, null_list=0.05, null_elem=0.05, max_len=4):
    lens = rng.integers(0, max_len, size=rows)
    nl = rng.random(rows) < null_list
    per = np.where((lens == 0) | nl, 1, lens)
    st = np.r_[0, np.cumsum(per)]
    rep = np.ones(int(st[-1]), np.uint8)
    rep[st[:-1]] = 0
    row_of = np.repeat(np.arange(rows), per)
    defs = np.where(rng.random(len(rep)) < null_elem, 2, 3).astype(np.uint8)
    defs[((lens == 0) & ~nl)[row_of]] = 1
    defs[nl[row_of]] = 0
    vals = rng.standard_normal(int((defs == 3).sum()))
    return defs, rep, vals


def test_oracle_list_closed_form():
    rng = np.random.default_rng(3)
    defs, rep, vals = _random_lists(rng, 5000)
    lv, lo, ev, evals, cnt = O.assemble_list(defs, rep, vals, 3, 1, 2, 8)
    starts = np.flatnonzero(rep == 0)
    el = defs >= 2
    assert np.array_equal(lo, np.r_[np.cumsum(el)[starts] - el[starts], el.sum()].astype(np.int32))
    assert np.array_equal(np.unpackbits(lv, bitorder="little")[:len(starts)].astype(bool), defs[starts] >= 1)
    ev_exp = defs[el] == 3
    assert np.array_equal(np.unpackbits(ev, bitorder="little")[:cnt[1]].astype(bool), ev_exp)
    spaced = np.zeros(cnt[1])
    spaced[ev_exp] = vals
    assert np.array_equal(evals.view(np.float64), spaced)


def _gpu_list(dec, defs, reps, vals, w):
    n = len(defs)
    dp = dec.upload(np.ascontiguousarray(defs, np.uint8))
    rp = dec.upload(np.ascontiguousarray(reps, np.uint8)) if reps is not None else None
    vp = dec.upload(np.ascontiguousarray(vals).view(np.uint8)) if w and len(vals) else (dec.upload(b"\0") if w else None)
    a, lvp, lop, evp, vvp = dec.assemble_list(dp, rp, vp, n, 3, 1, 2, w, values=w > 0)
    rows, el = a.num_rows, a.num_elements
    got = (dec.d2h(lvp, (rows + 7) // 8), dec.d2h(lop, (rows + 1) * 4, np.int32), dec.d2h(evp, (el + 7) // 8),
           dec.d2h(vvp, el * w) if w else np.zeros(0, np.uint8), (a.num_rows, a.num_elements, a.num_valid, a.null_lists))
    for p in (dp, rp, vp, lvp, lop, evp, vvp):
        if p:
            dec.free(p)
    return got


def _check_list(got, exp):
    for k, name in enumerate(("list validity", "list offsets", "element validity", "element values")):
        assert np.array_equal(got[k], exp[k]), name
    assert tuple(got[4]) == tuple(exp[4]), "counts"


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [0, 1, 40, 2000, 3001, 250_000, 3_000_000])
def test_gpu_list_export_random(dec, rows):
    rng = np.random.default_rng(rows + 1)
    defs, rep, vals = _random_lists(rng, rows, null_list=0.1, null_elem=0.2)
    exp = O.assemble_list(defs, rep, vals, 3, 1, 2, 8)
    _check_list(_gpu_list(dec, defs, rep, vals, 8), exp)


@pytest.mark.gpu
def test_gpu_list_export_malformed_levels(dec):
    """Unvalidated levels (Q6): leading rep > 0 slots, rep > 0 with def < elem_def."""
    rng = np.random.default_rng(9)
    n = 20_000
    defs = rng.integers(0, 4, size=n).astype(np.uint8)
    rep = rng.integers(0, 2, size=n).astype(np.uint8)
    rep[:5] = 1
    vals = rng.standard_normal(int((defs == 3).sum()))
    exp = O.assemble_list(defs, rep, vals, 3, 1, 2, 8)
    _check_list(_gpu_list(dec, defs, rep, vals, 8), exp)


@pytest.mark.gpu
def test_gpu_list_export_decoded_c5(dec):
    """Decode C5's LIST<double> chunk on the GPU, export it on the GPU, and match
    the oracle's decode + export (itself pinned to pyarrow above)."""
    import pqgpu
    data, pf, ch = _c5_list_chunk(rows=60_000, rg=7)
    devp = dec.upload(pf.data)
    try:
        r = dec.decode_jobs([pqgpu.device_job(pf, 0, 0, devp)])[0]
        assert r.status == 0
        a, lvp, lop, evp, vvp = dec.assemble_list(r.def_levels, r.rep_levels, r.values, r.num_slots, 3, 1, 2, 8)
        rows, el = a.num_rows, a.num_elements
        got = (dec.d2h(lvp, (rows + 7) // 8), dec.d2h(lop, (rows + 1) * 4, np.int32), dec.d2h(evp, (el + 7) // 8),
               dec.d2h(vvp, el * 8), (a.num_rows, a.num_elements, a.num_valid, a.null_lists))
        _check_list(got, O.assemble_list(ch.def_levels, ch.rep_levels, ch.values, 3, 1, 2, 8))
        assert rows == 60_000 and a.num_valid == r.num_values
        for p in (lvp, lop, evp, vvp):
            dec.free(p)
    finally:
        dec.free(devp)
