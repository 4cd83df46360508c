"""CPU oracle (oracle/liboracle.so) pinned against the reference's own vectors.

- bitpack32/64.json: unpack8int32Tests / unpack8int64Tests (bitpacking32_test.go,
  bitpacking64_test.go) — exact bytes <-> values, every width.
- crash_files.json: the reference's fuzz-crash regression files — must end in
  an error or a clean end, never a crash.
- round trips (hybrid_test.go / deltabp_test.go style) and an independent
  cross-check of whole files against pyarrow (this container only).
"""
import json
import os

import numpy as np
import pytest

import pqtest_util as U
from gen import pqwrite as W
from oracle import pyoracle as O
from pqgpu import abi

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_bitpack32_golden():
    vec = json.load(open(os.path.join(GOLD, "bitpack32.json")))["vectors"]
    assert len(vec) == 127
    for v in vec:
        got = O.unpack8(bytes.fromhex(v["data"]), v["width"], 32)
        assert got.tolist() == v["values"], v


def test_bitpack64_golden():
    vec = json.load(open(os.path.join(GOLD, "bitpack64.json")))["vectors"]
    assert len(vec) > 300
    for v in vec:
        got = O.unpack8(bytes.fromhex(v["data"]), v["width"], 64)
        assert got.tolist() == v["values"], v


@pytest.mark.parametrize("width", list(range(0, 33)))
def test_hybrid_roundtrip(width):
    rng = np.random.default_rng(width)
    hi = (1 << width) if width < 32 else (1 << 32)
    for n, runs in ((8 * 1024 + 5, False), (1000, True), (7, False)):
        if runs:
            v = np.repeat(rng.integers(0, hi, size=n // 10 + 1, dtype=np.uint64), 10)[:n]
        else:
            v = rng.integers(0, hi, size=n, dtype=np.uint64)
        v = v.astype(np.uint32)
        enc = W.hybrid_encode(v, width)
        rc, got = O.hybrid_decode(enc, width, n)
        assert rc == 0
        assert np.array_equal(got.view(np.uint32), v)


def test_hybrid_errors():
    # empty bit-packed run / empty RLE run (hybrid_decoder.go:143-166)
    assert O.hybrid_decode(b"\x01", 3, 1)[0] == -6
    assert O.hybrid_decode(b"\x00\x01", 3, 1)[0] == -6
    # RLE value too large for the width
    assert O.hybrid_decode(b"\x04\x09", 3, 2)[0] == -6
    # exhausted stream -> EOF
    assert O.hybrid_decode(b"\x04\x01", 3, 3)[0] == -1
    # short bit-packed group is zero padded (Q5): 1 group of width 8 with 3 bytes present
    rc, got = O.hybrid_decode(b"\x03\x01\x02\x03", 8, 8)
    assert rc == 0 and got.tolist() == [1, 2, 3, 0, 0, 0, 0, 0]
    # bit-packed group starting at EOF -> error
    assert O.hybrid_decode(b"\x05\x01\x02\x03\x04\x05\x06\x07\x08", 8, 9)[0] == -1
    # width 0: infinite zeros, reads nothing
    rc, got = O.hybrid_decode(b"", 0, 5)
    assert rc == 0 and got.tolist() == [0] * 5


@pytest.mark.parametrize("bits", [32, 64])
def test_delta_roundtrip(bits):
    rng = np.random.default_rng(bits)
    for n in (8 * 1024 + 5, 1000, 2, 130, 128 * 3 + 2):
        if bits == 64:
            v = rng.integers(-2**62, 2**62, size=n, dtype=np.int64)
        else:
            v = rng.integers(-2**31, 2**31 - 1, size=n, dtype=np.int64).astype(np.int32)
        enc = W.dbp_encode(v, bits)
        rc, got = O.delta_decode(enc, n, bits)
        assert rc == 0, n
        assert np.array_equal(got, v), n


def test_delta_q3():
    """Q3: N == 1 and (N-1) % 128 == 0 pages cannot be read back (deltabp_decoder.go:114-175)."""
    for n in (1, 129, 257):
        v = np.arange(n, dtype=np.int64) * 3
        enc = W.dbp_encode(v, 64)
        rc, _ = O.delta_decode(enc, n, 64)
        assert rc == -1, n
    v = np.arange(130, dtype=np.int64)
    assert O.delta_decode(W.dbp_encode(v, 64), 130, 64)[0] == 0


def test_snappy_against_pyarrow():
    import pyarrow as pa
    rng = np.random.default_rng(7)
    for data in (b"", b"a" * 100000, rng.integers(0, 4, size=70000, dtype=np.uint8).tobytes(),
                 rng.integers(0, 256, size=5000, dtype=np.uint8).tobytes(),
                 (b"lorem ipsum dolor sit amet " * 3000)):
        comp = pa.compress(data, codec="snappy", asbytes=True)
        rc, got = O.snappy_decode(comp, len(data) + 16)
        assert rc == 0 and got == data
        mine = W.snappy_compress(data)
        assert pa.decompress(mine, decompressed_size=len(data), codec="snappy", asbytes=True) == data
        rc, got = O.snappy_decode(mine, len(data) + 16)
        assert rc == 0 and got == data


def test_snappy_corrupt():
    assert O.snappy_decode(b"\x05\x10abc")[0] == -5       # literal longer than input
    assert O.snappy_decode(b"\x04\x01\x00")[0] == -5       # copy with offset 0 / before start
    assert O.snappy_decode(b"\xff\xff\xff\xff\xff\xff")[0] == -5


def _decode_file(data):
    import pqgpu
    pf = pqgpu.ParquetFile(data)
    out = []
    for rg in range(pf.num_row_groups):
        for c in range(pf.num_columns):
            job, _ = pf.host_job(rg, c)
            out.append((rg, c, O.decode_chunk(job)))
    return pf, out


def _check_against_arrow(data, np_dtype, col=0):
    pf, res = _decode_file(data)
    vals = np.concatenate([r.values.view(np_dtype) for (_, c, r) in res if c == col])
    for (_, c, r) in res:
        assert r.status == 0, abi.status_name(r.status)
    exp = U.dense_values(U.arrow_column(data, col), np_dtype)
    assert np.array_equal(vals, exp)
    return res


def test_c1_small_against_arrow():
    data, _ = W.config_c1(rows=50_000, rows_per_page=3000)
    res = _check_against_arrow(data, np.int64)
    assert len(res[0][2].pages) == 17


@pytest.mark.parametrize("bits", [0, 1, 2, 4, 8, 12, 16, 20])
@pytest.mark.parametrize("run_heavy", [False, True])
def test_c2_small_against_arrow(bits, run_heavy):
    data, info = W.config_c2(rows=40_000, bits=bits, run_heavy=run_heavy, rows_per_page=7000)
    res = _check_against_arrow(data, np.int32)
    r = res[0][2]
    assert r.num_values == info["non_null"]
    exp_def = ~np.asarray(U.arrow_column(data).combine_chunks().is_null())
    assert np.array_equal(r.def_levels.astype(bool), exp_def)


def test_c2_v2_snappy_against_arrow():
    data, info = W.config_c2(rows=30_000, bits=8, page_version=2, codec=W.SNAPPY, rows_per_page=4000)
    _check_against_arrow(data, np.int32)


def test_c3_small_against_arrow():
    data, _ = W.config_c3(rows=60_000, rows_per_page=20000)
    _check_against_arrow(data, np.int64)


def test_c3_int32_delta():
    rng = np.random.default_rng(11)
    v = rng.integers(-2**31, 2**31 - 1, size=30000, dtype=np.int64).astype(np.int32)
    col = W.Column("d32", W.INT32, v, encoding=W.DELTA_BINARY_PACKED, rows_per_page=5000, codec=W.SNAPPY,
                   page_version=2)
    data = W.write_file([col], len(v))
    _check_against_arrow(data, np.int32)


def test_plain_types_against_arrow():
    rng = np.random.default_rng(5)
    n = 5000
    f32 = rng.standard_normal(n).astype(np.float32)
    f32[::97] = np.nan
    f64 = rng.standard_normal(n)
    i96 = rng.integers(0, 256, size=n * 12, dtype=np.uint8)
    cols = [W.Column("f", W.FLOAT, f32, rows_per_page=1000), W.Column("d", W.DOUBLE, f64, rows_per_page=999),
            W.Column("b", W.BOOLEAN, rng.integers(0, 2, n).astype(np.uint8), rows_per_page=1001),
            W.Column("fx", W.FLBA, rng.integers(0, 256, size=n * 5, dtype=np.uint8), type_length=5,
                     rows_per_page=700),
            W.Column("i96", W.INT96, i96, rows_per_page=333)]
    data = W.write_file(cols, n)
    pf, res = _decode_file(data)
    for (_, c, r) in res:
        assert r.status == 0
    assert res[0][2].values.view(np.float32).view(np.uint32).tolist() == f32.view(np.uint32).tolist()
    assert np.array_equal(res[1][2].values.view(np.float64), f64)
    assert np.array_equal(res[2][2].values, cols[2].values)
    assert np.array_equal(res[3][2].values, cols[3].values)
    assert np.array_equal(res[4][2].values, i96)


def test_c4_small_against_arrow():
    data, _ = W.config_c4(rows=30_000, vocab=4000, dict_limit=40 << 10, rows_per_page=1500)
    pf, res = _decode_file(data)
    r = res[0][2]
    assert r.status == 0
    offs = r.offsets
    got = [r.values[offs[i]:offs[i + 1]].tobytes() for i in range(r.num_values)]
    exp = [x.as_py() for x in U.arrow_column(data).combine_chunks()]
    exp = [e.encode() if isinstance(e, str) else e for e in exp]
    assert got == exp
    encs = {p.encoding for p in r.pages if p.page_type == 0}
    assert encs == {0, 8}, encs  # dictionary pages then PLAIN fallback


def test_list_levels_against_arrow():
    rng = np.random.default_rng(9)
    rows = 3000
    lens = rng.integers(0, 4, size=rows)
    null_list = rng.random(rows) < 0.05
    rep, defs, vals = [], [], []
    for r in range(rows):
        if null_list[r]:
            rep.append(0); defs.append(0)
        elif lens[r] == 0:
            rep.append(0); defs.append(1)
        else:
            for k in range(lens[r]):
                rep.append(0 if k == 0 else 1)
                if rng.random() < 0.05:
                    defs.append(2)
                else:
                    defs.append(3)
                    vals.append(rng.standard_normal())
    col = W.Column("l", W.DOUBLE, np.array(vals), repetition=W.LIST, def_levels=np.array(defs),
                   rep_levels=np.array(rep), rows_per_page=500)
    data = W.write_file([col], rows)
    pf, res = _decode_file(data)
    r = res[0][2]
    assert r.status == 0 and pf.columns[0].desc.max_def == 3 and pf.columns[0].desc.max_rep == 1
    assert r.rep_levels.tolist() == rep and r.def_levels.tolist() == defs
    assert np.array_equal(r.values.view(np.float64), np.array(vals))
    a = U.arrow_column(data).combine_chunks()
    assert a.to_pylist()[:50] == [None if null_list[i] else [None if False else x for x in a[i].as_py()]
                                  for i in range(50)]


def test_dremel_twitter_levels():
    """TestTwitterBlog (data_store_test.go:346-389): rep/def level vectors of a
    two-level repeated column decode back exactly from a hand-built V1 page."""
    g = json.load(open(os.path.join(GOLD, "dremel.json")))
    rep = W.hybrid_encode(g["rep_levels"], 2)
    defs = W.hybrid_encode(g["def_levels"], 2)
    vals = np.array(g["values"], dtype=np.int32).tobytes()
    page = U.v1_page(vals, len(g["rep_levels"]), 0, rep=rep, defs=defs)
    keep = []
    job, _ = U.chunk_job(page, abi.INT32, max_def=2, max_rep=2, keep=keep)
    r = O.decode_chunk(job)
    assert r.status == 0
    assert r.rep_levels.tolist() == g["rep_levels"]
    assert r.def_levels.tolist() == g["def_levels"]
    assert r.values.view(np.int32).tolist() == g["values"]


def test_crash_files_never_crash():
    import pqgpu
    files = json.load(open(os.path.join(GOLD, "crash_files.json")))["files"]
    assert len(files) == 8
    for f in files:
        data = bytes.fromhex(f["data"])
        try:
            pf = pqgpu.ParquetFile(data)
        except pqgpu.PqgError:
            continue  # NewFileReader returned an error: acceptable outcome
        for rg in range(pf.num_row_groups):
            for c in range(pf.num_columns):
                try:
                    job, _ = pf.host_job(rg, c)
                except pqgpu.PqgError:
                    continue
                O.decode_chunk(job)  # any status is fine; must not crash


def test_c5_columns_against_arrow():
    """C5 (two row groups): every flat column's oracle decode equals pyarrow's."""
    import pyarrow as pa
    data, _ = W.config_c5(row_groups=(2, 9), rows_per_rg=20_000)
    pf, res = _decode_file(data)
    assert all(r.status == 0 for (_, _, r) in res)
    dt = {1: np.int32, 2: np.int64, 3: np.int64, 4: np.float32, 5: np.float64}
    for c in range(1, pf.num_columns):
        name = pf.columns[c].path.decode()
        parts = [r for (_, cc, r) in res if cc == c]
        arr = U.arrow_column(data, c).combine_chunks()
        if name == "s":
            got = []
            for r in parts:
                got += [r.values[r.offsets[i]:r.offsets[i + 1]].tobytes() for i in range(r.num_values)]
            assert got == [x.as_py().encode() for x in arr]
        elif name == "i96":
            # pyarrow converts INT96 to timestamps; compare the raw 12-byte values with the generator's
            rg_cols = [W.c5_row_group_columns(rg, 20_000)["i96"]["values"] for rg in (2, 9)]
            assert np.array_equal(np.concatenate([r.values for r in parts]), np.concatenate(rg_cols))
        else:
            t = dt[pf.columns[c].desc.physical_type]
            got = np.concatenate([r.values.view(t) for r in parts])
            exp = U.dense_values(U.arrow_column(data, c), t)
            assert np.array_equal(got.view(np.uint8), exp.view(np.uint8)), name
            if name == "oi32":
                defs = np.concatenate([r.def_levels for r in parts]).astype(bool)
                assert np.array_equal(defs, np.asarray(arr.is_valid()))
    assert isinstance(pa.__version__, str)
