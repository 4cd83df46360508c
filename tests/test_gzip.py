"""GZIP pages (gzipCompressor.DecompressBlock, compress.go:63-76, registered at
compress.go:152-156): the oracle decodes them with Go's compress/gzip
semantics (multistream members until the block ends; zlib for DEFLATE).

The reference's own tests only round-trip gzip (compress_test.go:11-32), so the
oracle is checked here against pyarrow-written GZIP files (an independent
writer and reader) and against hand-built pages: two concatenated members
(Go's default multistream mode reads both), a corrupt member, trailing
garbage, a truncated member."""
import gzip
import io
import zlib

import numpy as np
import pytest

import pqtest_util as U
from oracle import pyoracle as O
from pqgpu import abi


def _pyarrow_gzip_file(version):
    pa = pytest.importorskip("pyarrow")
    pq = pytest.importorskip("pyarrow.parquet")
    rng = np.random.default_rng(31)
    n = 30000
    words = ["g%04d" % i for i in range(300)]
    t = pa.table({
        "i64": pa.array(rng.integers(-2**40, 2**40, n)),
        "f64": pa.array(rng.standard_normal(n)),
        "o32": pa.array([int(x) if x % 7 else None for x in rng.integers(0, 1000, n)], type=pa.int32()),
        "s": pa.array([words[int(i)] for i in rng.integers(0, 300, n)]),
    })
    buf = io.BytesIO()
    pq.write_table(t, buf, compression="gzip", data_page_version=version, data_page_size=64 * 1024,
                   use_dictionary=["s", "o32"])
    return buf.getvalue(), t


@pytest.mark.parametrize("version", ["1.0"])
def test_oracle_pyarrow_gzip_file(version):
    import pqgpu
    data, t = _pyarrow_gzip_file(version)
    pf = pqgpu.ParquetFile(data)
    for c in range(pf.num_columns):
        assert pf.chunk_meta(0, c).codec == abi.CODEC_GZIP
        r = O.decode_chunk(pf.host_job(0, c)[0])
        assert r.status == 0, abi.status_name(r.status)
        col = t.column(c).combine_chunks()
        vals = col.drop_null() if hasattr(col, "drop_null") else col.filter(col.is_valid())
        if c == 3:
            offs = np.asarray(r.offsets)
            got = [bytes(np.asarray(r.values)[offs[i]:offs[i + 1]]).decode() for i in range(len(offs) - 1)]
            assert got == vals.to_pylist()
        else:
            dt = {0: np.int64, 1: np.float64, 2: np.int32}[c]
            assert np.array_equal(np.asarray(r.values).view(dt), np.asarray(vals.to_numpy()).astype(dt))


def _gz_page(body_plain, gz_bytes, nvals):
    hdr = U.page_header_v1(len(body_plain), len(gz_bytes), nvals, abi.ENC_PLAIN)
    return hdr + gz_bytes


def _decode(chunk):
    job, _ = U.chunk_job(chunk, ptype=abi.INT64, codec=abi.CODEC_GZIP)
    return O.decode_chunk(job)


def test_oracle_gzip_members():
    v = np.arange(5000, dtype=np.int64) * 3
    raw = v.tobytes()
    one = gzip.compress(raw)
    r = _decode(_gz_page(raw, one, len(v)))
    assert r.status == 0 and np.array_equal(np.asarray(r.values).view(np.int64), v)
    # two members (gzip.Reader multistream mode): their bytes concatenated
    two = gzip.compress(raw[:16000]) + gzip.compress(raw[16000:])
    r = _decode(_gz_page(raw, two, len(v)))
    assert r.status == 0 and np.array_equal(np.asarray(r.values).view(np.int64), v)


@pytest.mark.parametrize("how", ["crc", "trailing", "truncated", "header", "empty"])
def test_oracle_gzip_errors(how):
    v = np.arange(3000, dtype=np.int64)
    raw = v.tobytes()
    gz = bytearray(gzip.compress(raw))
    if how == "crc":
        gz[-8] ^= 1                 # CRC-32 of the member
    elif how == "trailing":
        gz += b"\x00\x01"           # not a member header after the member
    elif how == "truncated":
        gz = gz[:-5]
    elif how == "header":
        gz[0] = 0x1e
    else:
        gz = bytearray()
    r = _decode(_gz_page(raw, bytes(gz), len(v)))
    assert r.status == abi.STATUS_CODES["GZIP"], abi.status_name(r.status)


def test_oracle_gzip_size_mismatch():
    raw = np.arange(100, dtype=np.int64).tobytes()
    page = U.page_header_v1(len(raw) + 8, len(gzip.compress(raw)), 100, abi.ENC_PLAIN) + gzip.compress(raw)
    r = _decode(page)
    assert r.status == abi.STATUS_CODES["SIZE"]
