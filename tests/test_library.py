"""CPU-side checks of the product library: it loads, exports every symbol the
C ABI header declares, and its host planner (footer + schema) works."""
import os
import re

import numpy as np

import pqgpu
from gen import pqwrite as W
from pqgpu import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols(prefix):
    text = open(os.path.join(ROOT, "include", "pqgpu.h")).read()
    return sorted(set(re.findall(r"\b(%s_[a-z0-9_]+)\s*\(" % prefix, text)))


def test_library_exports_header_symbols():
    L = _lib.lib()
    syms = header_symbols("pqg")
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(_lib.EXPORTED) == sorted(syms)


def test_oracle_exports_header_symbols():
    from oracle import pyoracle
    L = pyoracle.lib()
    for s in header_symbols("pqo"):
        assert hasattr(L, s), s


def test_product_does_not_link_oracle():
    import subprocess
    out = subprocess.run(["ldd", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out
    nm = subprocess.run(["nm", "-D", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "pqo_" not in nm


def test_planner_schema_levels():
    rng = np.random.default_rng(1)
    n = 1000
    cols = [W.Column("req", W.INT64, rng.integers(0, 9, n)),
            W.Column("opt", W.INT32, rng.integers(0, 9, n).astype(np.int32)[: n - 10], repetition=W.OPTIONAL,
                     def_levels=np.r_[np.ones(n - 10), np.zeros(10)].astype(np.uint8)),
            W.Column("lst", W.DOUBLE, np.arange(n, dtype=np.float64), repetition=W.LIST,
                     def_levels=np.full(n, 3), rep_levels=np.zeros(n))]
    data = W.write_file(cols, n, row_groups=3)
    pf = pqgpu.ParquetFile(data)
    assert pf.num_columns == 3 and pf.num_row_groups == 3 and pf.num_rows == n
    d = [(c.path.decode(), c.desc.max_def, c.desc.max_rep) for c in pf.columns]
    assert d == [("req", 0, 0), ("opt", 1, 0), ("lst.list.element", 3, 1)]
    m = pf.chunk_meta(1, 2)
    assert m.total_compressed_size > 0 and m.num_values == 334


def test_planner_rejects_bad_footer():
    import pytest
    for bad in (b"", b"PAR1", b"PAR1xxxxPAR1", b"PAR1" + b"\x00" * 8 + b"\xff\xff\xff\x7fPAR1"):
        with pytest.raises(pqgpu.PqgError):
            pqgpu.ParquetFile(bad)


UNSIGNED = [("u32", 1, 1), ("u64", 1, 2), ("i32", 0, 1), ("u8", 1, 1), ("i64", 0, 2)]


def test_planner_unsigned_flag():
    """pqg_column_desc.flags bit0 is getInt32ValuesDecoder's / getInt64ValuesDecoder's
    unSigned (ConvertedType UINT_8/16/32/64 or INTEGER(isSigned=false),
    chunk_reader.go:99-141), and the oracle echoes it into the result."""
    from oracle import pyoracle as O
    data = open(os.path.join(ROOT, "tests", "golden", "unsigned.parquet"), "rb").read()
    pf = pqgpu.ParquetFile(data)
    got = [(c.path.decode(), c.desc.flags & 1, c.desc.physical_type) for c in pf.columns]
    assert got == UNSIGNED
    for i in range(pf.num_columns):
        ch = O.decode_chunk(pf.host_job(0, i)[0])
        assert ch.status == 0 and ch.col_flags == pf.columns[i].desc.flags


def test_planner_footer_only_open(tmp_path):
    """pqg_file_open_tail (readFileMetaData file_meta.go:14-62 from the head and
    the footer only) plans exactly what pqg_file_open plans from the whole file;
    a range reader's chunk spans cover only the selected chunks."""
    data, _ = W.config_c5(row_groups=(0, 1, 2), rows_per_rg=2000, rows_per_page=700)
    path = tmp_path / "f.parquet"
    path.write_bytes(data)
    a, b = pqgpu.ParquetFile(data), pqgpu.ParquetFile.open(str(path))
    assert (a.num_columns, a.num_row_groups, a.num_rows) == (b.num_columns, b.num_row_groups, b.num_rows)
    for rg in range(3):
        for c in range(a.num_columns):
            assert bytes(a.chunk_meta(rg, c)) == bytes(b.chunk_meta(rg, c))
            m = b.chunk_meta(rg, c)
            assert bytes(b.read_range(m.start, m.start + m.total_compressed_size)) == \
                data[m.start:m.start + m.total_compressed_size]
    lo, hi, _ = pqgpu.chunk_span(b, [(1, c) for c in range(b.num_columns)])
    assert 4 < lo and hi < b.size - 8  # row group 1 alone: neither neighbour is read
    L = _lib.lib()
    import ctypes as C
    h = C.c_void_p()
    assert L.pqg_file_open_tail(data[:4], 4, data[-8:], 8, len(data), C.byref(h)) == \
        pqgpu.abi.STATUS_CODES["INVALID_ARG"]  # the tail must hold the footer
    assert L.pqg_file_open_tail(b"PAR2", 4, data, len(data), len(data), C.byref(h)) == \
        pqgpu.abi.STATUS_CODES["METADATA"]
