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


@pytest.mark.parametrize("version", ["1.0", "2.0"])
def test_oracle_pyarrow_gzip_file(version):
    import pqgpu
    data, t = _pyarrow_gzip_file(version)
    pf = pqgpu.ParquetFile(data)
    for c in range(pf.num_columns):
        assert pf.chunk_meta(0, c).codec == abi.CODEC_GZIP
        r = O.decode_chunk(pf.host_job(0, c)[0])
        if version == "2.0" and c == 2:
            # pyarrow stores this V2 page raw with is_compressed=false (its
            # gzip body would be larger); the reference ignores the flag and
            # gunzips it anyway (Q4, page_v2.go:110-123)
            assert r.status == abi.STATUS_CODES["GZIP"] and r.error_page == 1
            continue
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


def test_oracle_gzip_block_api():
    raw = np.arange(4000, dtype=np.int64).tobytes()
    assert O.gzip_decode(gzip.compress(raw)) == (0, raw)
    assert O.gzip_decode(gzip.compress(raw) + gzip.compress(b"xy")) == (0, raw + b"xy")
    assert O.gzip_decode(b"12345")[0] == abi.STATUS_CODES["GZIP"]


# ---- K2g: the GPU inflate kernel (pqg_inflate.hip) vs the oracle ------------

def _zlib_gzip(raw, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, mem=8):
    c = zlib.compressobj(level, zlib.DEFLATED, 31, mem, strategy)
    return c.compress(raw) + c.flush()


def _gz_with_header_fields(raw):
    """A member with FEXTRA, FNAME, FCOMMENT and FHCRC (RFC 1952 2.3.1)."""
    body = zlib.compressobj(6, zlib.DEFLATED, -15)
    deflate = body.compress(raw) + body.flush()
    flg = 0x04 | 0x08 | 0x10 | 0x02
    hdr = bytes([0x1f, 0x8b, 8, flg, 0, 0, 0, 0, 0, 3])
    hdr += (5).to_bytes(2, "little") + b"xtra!" + b"name.bin\0" + b"a comment\0"
    hdr += (zlib.crc32(hdr) & 0xffff).to_bytes(2, "little")
    return hdr + deflate + (zlib.crc32(raw) & 0xffffffff).to_bytes(4, "little") + \
        (len(raw) & 0xffffffff).to_bytes(4, "little")


def _gz_named(raw, name_len, comment_len=0):
    """A member whose FNAME (and FCOMMENT) hold name_len (comment_len) bytes before the NUL."""
    body = zlib.compressobj(6, zlib.DEFLATED, -15)
    deflate = body.compress(raw) + body.flush()
    flg = 0x08 | (0x10 if comment_len else 0)
    hdr = bytes([0x1f, 0x8b, 8, flg, 0, 0, 0, 0, 0, 3]) + b"n" * name_len + b"\0"
    if comment_len:
        hdr += b"c" * comment_len + b"\0"
    return hdr + deflate + (zlib.crc32(raw) & 0xffffffff).to_bytes(4, "little") + \
        (len(raw) & 0xffffffff).to_bytes(4, "little")


# Go's compress/gzip readString reads FNAME / FCOMMENT into a [512]byte buffer:
# 511 bytes + the NUL decode, 512 bytes before the NUL fail with ErrHeader
NAME_CASES = [(511, 0, 0), (512, 0, "GZIP"), (0, 511, 0), (3, 512, "GZIP"), (2000, 0, "GZIP")]


@pytest.mark.parametrize("name_len,comment_len,want", NAME_CASES)
def test_oracle_gzip_name_bound(name_len, comment_len, want):
    raw = b"hello parquet " * 50
    rc, out = O.gzip_decode(_gz_named(raw, name_len, comment_len))
    assert rc == (abi.STATUS_CODES[want] if want else 0)
    if not want:
        assert out == raw


def _gpu_blocks():
    rng = np.random.default_rng(44)
    rep = np.repeat(rng.integers(0, 50, 40000), rng.integers(1, 30, 40000)).astype(np.int64).tobytes()
    text = b" ".join(b"w%d" % int(i) for i in rng.integers(0, 3000, 200000))
    noise = rng.integers(0, 256, 300000, dtype=np.uint8).tobytes()
    return {
        "dynamic": (rep, gzip.compress(rep)),
        "text": (text, _zlib_gzip(text, 9)),
        "stored": (noise, gzip.compress(noise)),
        "level0": (text[:200000], _zlib_gzip(text[:200000], 0)),
        "fixed": (rep[:300000], _zlib_gzip(rep[:300000], 6, zlib.Z_FIXED)),
        "rle": (bytes(500000), _zlib_gzip(bytes(500000), 9, zlib.Z_RLE)),
        "huffonly": (text[:100000], _zlib_gzip(text[:100000], 6, zlib.Z_HUFFMAN_ONLY)),
        "small_window": (text, _zlib_gzip(text, 6, mem=1)),
        "members": (rep + text, gzip.compress(rep) + gzip.compress(text)),
        "header_fields": (text[:50000], _gz_with_header_fields(text[:50000])),
        "empty": (b"", gzip.compress(b"")),
        "one": (b"z", gzip.compress(b"z")),
    }


@pytest.fixture(scope="module")
def dec():
    import pqgpu
    d = pqgpu.GpuDecoder(0)
    yield d
    d.close()


def _gpu_block(dec, src, cap):
    import ctypes as C
    dst = np.zeros(max(cap, 1), np.uint8)
    n = C.c_int64(0)
    rc = dec.L.pqg_block_decompress(dec.ctx, abi.CODEC_GZIP, src, len(src), dst.ctypes.data, cap, C.byref(n))
    return rc, n.value, dst


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(_gpu_blocks().keys()))
def test_gpu_inflate_block(dec, name):
    raw, gz = _gpu_blocks()[name]
    assert O.gzip_decode(gz) == (0, raw)
    rc, n, dst = _gpu_block(dec, gz, len(raw) + 100)
    assert rc == 0, abi.status_name(rc)
    assert n == len(raw) and dst[:n].tobytes() == raw
    if raw:  # a too small output buffer: the length, nothing written
        rc, n, _ = _gpu_block(dec, gz, len(raw) - 1)
        assert rc == abi.ERR_CAPACITY and n == len(raw)


@pytest.mark.gpu
@pytest.mark.parametrize("how", ["crc", "isize", "trailing", "truncated", "header", "empty", "method", "bad_block",
                                 "distance", "hcrc"])
def test_gpu_inflate_block_errors(dec, how):
    raw = np.arange(30000, dtype=np.int64).tobytes()
    gz = bytearray(gzip.compress(raw))
    if how == "crc":
        gz[-8] ^= 1
    elif how == "isize":
        gz[-1] ^= 1
    elif how == "trailing":
        gz += b"\x00\x01"
    elif how == "truncated":
        gz = gz[:-5]
    elif how == "header":
        gz[0] = 0x1e
    elif how == "empty":
        gz = bytearray()
    elif how == "method":
        gz[2] = 7
    elif how == "bad_block":
        gz[10] |= 0x06  # BTYPE 3 (reserved) in the first block header
    elif how == "distance":  # a fixed-Huffman block whose first code is a match (nothing behind it)
        body = bytes([0x03 | (0x01 << 3), 0x00, 0x00]) + b"\x00" * 4
        gz = bytearray(gz[:10] + body + gz[-8:])
    else:  # FHCRC with a wrong header CRC-16
        gz = bytearray(_gz_with_header_fields(raw))
        gz[10 + 2 + 5 + 9 + 10] ^= 0xff
    rc_o, _ = O.gzip_decode(bytes(gz))
    assert rc_o == abi.STATUS_CODES["GZIP"]
    rc, _, _ = _gpu_block(dec, bytes(gz), len(raw) + 64)
    assert rc == rc_o, (abi.status_name(rc), abi.status_name(rc_o))


@pytest.mark.gpu
@pytest.mark.parametrize("version", ["1.0", "2.0"])
def test_gpu_pyarrow_gzip_file(dec, version):
    import parity as P
    data, _ = _pyarrow_gzip_file(version)
    P.compare_file(data, dec)


@pytest.mark.gpu
def test_gpu_gzip_many_pages(dec):
    """Many GZIP pages in one batch (the inflate queue), every writer layout."""
    import parity as P
    pa = pytest.importorskip("pyarrow")
    pq = pytest.importorskip("pyarrow.parquet")
    rng = np.random.default_rng(32)
    n = 400_000
    t = pa.table({"a": pa.array(rng.integers(0, 1 << 20, n)),
                  "b": pa.array(np.repeat(rng.standard_normal(n // 8), 8)),
                  "c": pa.array([None if x % 5 == 0 else int(x) for x in rng.integers(0, 40, n)], type=pa.int32())})
    buf = io.BytesIO()
    pq.write_table(t, buf, compression="gzip", data_page_size=16 * 1024, row_group_size=150_000)
    P.compare_file(buf.getvalue(), dec)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["members", "stored", "fixed", "header_fields", "one"])
def test_gpu_gzip_hand_pages(dec, name):
    import parity as P
    raw, gz = _gpu_blocks()[name]
    raw = raw[: len(raw) // 8 * 8]
    if len(raw) == 0:
        raw = np.arange(1, dtype=np.int64).tobytes()
    gz = {"members": gzip.compress(raw[:8000]) + gzip.compress(raw[8000:]), "stored": gzip.compress(raw),
          "fixed": _zlib_gzip(raw, 6, zlib.Z_FIXED), "header_fields": _gz_with_header_fields(raw),
          "one": gzip.compress(raw)}[name]
    exp, _ = P.compare_chunk_bytes(_gz_page(raw, gz, len(raw) // 8), dec, ptype=abi.INT64, codec=abi.CODEC_GZIP)
    assert exp.status == 0


@pytest.mark.gpu
@pytest.mark.parametrize("how", ["crc", "trailing", "truncated", "size"])
def test_gpu_gzip_page_errors(dec, how):
    import parity as P
    raw = np.arange(3000, dtype=np.int64).tobytes()
    gz = bytearray(gzip.compress(raw))
    ulen = len(raw)
    if how == "crc":
        gz[-8] ^= 1
    elif how == "trailing":
        gz += b"\x00\x01"
    elif how == "truncated":
        gz = gz[:-5]
    else:
        ulen += 8
    page = U.page_header_v1(ulen, len(gz), 3000, abi.ENC_PLAIN) + bytes(gz)
    exp, _ = P.compare_chunk_bytes(page, dec, ptype=abi.INT64, codec=abi.CODEC_GZIP)
    assert exp.status != 0


@pytest.mark.gpu
@pytest.mark.parametrize("name_len,comment_len,want", NAME_CASES)
def test_gpu_gzip_name_bound(dec, name_len, comment_len, want):
    raw = b"hello parquet " * 50
    rc, n, dst = _gpu_block(dec, _gz_named(raw, name_len, comment_len), len(raw) + 16)
    assert rc == (abi.STATUS_CODES[want] if want else 0), abi.status_name(rc)
    if not want:
        assert dst[:n].tobytes() == raw


REDO = 64  # PQG_PAGE_FLAG_INFLATE_REDO


def _far_raw(n=12000, reps=3, seed=45):
    """Random bytes repeated: every match reaches n bytes back, past the 8 KiB ring."""
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, n, dtype=np.uint8).tobytes() * reps


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["far", "far_near", "text_window", "far_members", "far_fixed"])
def test_gpu_gzip_far_matches(dec, name):
    """k_inflate_s keeps 8 KiB of history in LDS; matches reaching further
    (up to the 32 KiB window) read their bytes back from the page's stored
    output.  Bit-exact against the oracle; no page needs the 32 KiB pass."""
    import parity as P
    rng = np.random.default_rng(46)
    far = _far_raw()
    raw = {"far": far,
           "far_near": b"".join(far[i:i + 3000] + bytes(rng.integers(0, 4, 500, dtype=np.uint8))
                                for i in range(0, 36000, 3000)),
           "text_window": b" ".join(b"v%d" % int(i) for i in rng.integers(0, 9000, 40000)),
           "far_members": far + far,
           "far_fixed": far}[name]
    raw = raw[: len(raw) // 8 * 8]
    gz = {"far_members": gzip.compress(far) + gzip.compress(far),
          "far_fixed": _zlib_gzip(raw, 6, zlib.Z_FIXED)}.get(name) or _zlib_gzip(raw, 9)
    exp, got = P.compare_chunk_bytes(_gz_page(raw, gz, len(raw) // 8), dec, ptype=abi.INT64, codec=abi.CODEC_GZIP)
    assert exp.status == 0
    assert not any(p.flags & REDO for p in got.pages)


@pytest.mark.gpu
@pytest.mark.parametrize("short", [8, 4000, 12008, 23992])
def test_gpu_gzip_far_match_past_size(dec, short):
    """A page that decodes to more than its uncompressed size: bytes past the
    size are never stored, so a far match reading one sends the page to the
    32 KiB-ring pass, which reports the same status as the oracle (SIZE)."""
    import parity as P
    raw = _far_raw()
    gz = _zlib_gzip(raw, 9)
    ulen = len(raw) - short
    page = U.page_header_v1(ulen, len(gz), ulen // 8, abi.ENC_PLAIN) + gz
    exp, got = P.compare_chunk_bytes(page, dec, ptype=abi.INT64, codec=abi.CODEC_GZIP)
    assert exp.status == abi.STATUS_CODES["SIZE"], abi.status_name(exp.status)
    # a far match reads bytes 12000 back: past the size when the size ends before 24000
    assert bool(any(p.flags & REDO for p in got.pages)) == (ulen < 24000)
