"""FileReader byte ranges (pqgpu.reader): chunks whose last page runs past an
understated TotalCompressedSize.

readPages (chunk_reader.go:206-284) reads page headers while
TotalCompressedSize - Count() > 0 and then reads each page whole from the file
(newBlockReader, compress.go:102-122), so a last page that starts inside the
declared size but ends past it decodes normally in parquet-go.  The planner
uploads only [start, start + TotalCompressedSize) per selected chunk;
decode_spans re-uploads such a chunk to the end of the file when its decode
ends in EOF / size mismatch.  The oracle (test infrastructure) reads a host job
over the whole file, like the reference."""
import numpy as np
import pytest

import pqtest_util as U  # noqa: F401  (sys.path)
import pqgpu
from gen import pqwrite as W
from oracle import pyoracle as O


def _file(rows=30_000):
    rng = np.random.default_rng(11)
    cols = [
        W.Column("a", W.INT64, rng.integers(-2**40, 2**40, size=rows, dtype=np.int64), rows_per_page=7000),
        W.Column("b", W.INT32, rng.integers(-2**31, 2**31 - 1, size=rows, dtype=np.int64).astype(np.int32),
                 rows_per_page=7000),
        W.Column("c", W.INT96, rng.integers(0, 256, size=rows * 12, dtype=np.uint8), rows_per_page=7000),
    ]
    return W.write_file(cols, rows)


def understate_tcs(data, rg, col, d):
    """The file with chunk (rg, col)'s TotalCompressedSize (and an equal
    TotalUncompressedSize, a hint) lowered by d in the thrift footer, the
    varint length kept."""
    pf = pqgpu.ParquetFile(data)
    tcs = pf.chunk_meta(rg, col).total_compressed_size
    old, new = U.zigzag(tcs), U.zigzag(tcs - d)
    assert len(old) == len(new)
    flen = int.from_bytes(data[-8:-4], "little")
    f0 = len(data) - 8 - flen
    buf = bytearray(data)
    hits = 0
    i = f0
    while True:
        i = bytes(buf).find(old, i + 1, len(data) - 8)
        if i < 0:
            break
        if buf[i - 1] & 0x0F == 6:  # an i64 field header (compact protocol) in front
            buf[i:i + len(old)] = new
            hits += 1
    assert hits >= 1
    out = bytes(buf)
    p2 = pqgpu.ParquetFile(out)
    assert p2.chunk_meta(rg, col).total_compressed_size == tcs - d
    for c in range(pf.num_columns):
        if c != col:
            assert p2.chunk_meta(rg, c).total_compressed_size == pf.chunk_meta(rg, c).total_compressed_size
    return out


def test_oracle_reads_the_last_page_past_tcs():
    data = _file()
    bad = understate_tcs(data, 0, 0, 5)
    a = O.decode_chunk(pqgpu.ParquetFile(data).host_job(0, 0)[0])
    b = O.decode_chunk(pqgpu.ParquetFile(bad).host_job(0, 0)[0])
    assert a.status == 0 and b.status == 0
    assert np.array_equal(a.values, b.values)


def test_chunk_ranges_to_eof():
    data = _file()
    pf = pqgpu.ParquetFile(data)
    specs = [(0, 0), (0, 2)]
    rs, metas = pqgpu.chunk_ranges(pf, specs)
    assert len(rs) == 2  # non-adjacent: column b is skipped
    rs2, _ = pqgpu.chunk_ranges(pf, specs, to_eof={0})
    m = metas[0]
    assert rs2[0][0] == m.start and rs2[-1][1] == pf.size


@pytest.mark.gpu
def test_file_reader_understated_tcs_projection(tmp_path):
    data = _file()
    bad = understate_tcs(data, 0, 0, 5)
    path = tmp_path / "bad.parquet"
    path.write_bytes(bad)
    fr = pqgpu.FileReader(str(path), "a", "c")
    try:
        got = fr.read_row_group(0)
        pf = pqgpu.ParquetFile(bad)
        for name, col in (("a", 0), ("c", 2)):
            exp = O.decode_chunk(pf.host_job(0, col)[0])
            assert exp.status == 0
            g = got[name]
            assert g.status == 0, name
            assert np.array_equal(g.values, exp.values), name
        # the retry uploaded column a's bytes to the end of the file
        m = pf.chunk_meta(0, 0)
        assert fr.uploaded_bytes > pf.size - m.start
    finally:
        fr.dec.close()
