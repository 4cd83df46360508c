"""DELTA_LENGTH_BYTE_ARRAY and DELTA_BYTE_ARRAY: the oracle's
restatement of byteArrayDeltaLengthDecoder / byteArrayDeltaDecoder
(type_bytearray.go:97-240, lengths through deltaBitPackDecoder32
deltabp_decoder.go:38-175) against the generator's own values and against
pyarrow (an independent writer and reader), the error classes of hand-built
pages, and (-m gpu) the GPU path (k_str_delta, k_str_copy, k_str_dba) against
the oracle on the same files, byte for byte.

The reference's own tests hold no vectors for these encodings (types_test.go
:189-214 only round-trips 2000 random values through its encoder): parity is
pinned by the format, by pyarrow, and by the quirks of the cited lines
(Q3: a one-value length stream has no miniblock, so init fails with EOF)."""
import io

import numpy as np
import pytest

import parity as P
import pqtest_util as U
from gen import pqwrite as W
from oracle import pyoracle as O
from pqgpu import abi

DLBA, DBA = W.DELTA_LENGTH_BYTE_ARRAY, W.DELTA_BYTE_ARRAY


def _strings(r):
    offs = np.asarray(r.offsets)
    v = np.asarray(r.values)
    return [bytes(v[offs[i]:offs[i + 1]]) for i in range(len(offs) - 1)]


def _expected(exp):
    offs, chars = exp["offsets"], exp["chars"]
    return [bytes(chars[offs[i]:offs[i + 1]]) for i in range(len(offs) - 1)]


CASES = [dict(encoding=e, page_version=v, codec=c, null_frac=nf, sorted_values=s)
         for e in (DLBA, DBA) for v in (1, 2) for c in (W.UNCOMPRESSED, W.SNAPPY)
         for nf, s in ((0.0, True), (0.15, False))]


@pytest.mark.parametrize("kw", CASES, ids=lambda k: "e%d_v%d_c%d_n%d_s%d" % (
    k["encoding"], k["page_version"], k["codec"], int(k["null_frac"] * 100), k["sorted_values"]))
def test_oracle_generated_files(kw):
    import pqgpu
    data, exp = W.config_delta_strings(rows=12000, rows_per_page=2500, **kw)
    pf = pqgpu.ParquetFile(data)
    r = O.decode_chunk(pf.host_job(0, 0)[0])
    assert r.status == 0, abi.status_name(r.status)
    assert _strings(r) == _expected(exp)
    if exp["defs"] is not None:
        assert np.array_equal(np.asarray(r.def_levels), exp["defs"])


@pytest.mark.parametrize("enc", ["DELTA_LENGTH_BYTE_ARRAY", "DELTA_BYTE_ARRAY"])
@pytest.mark.parametrize("version", ["1.0", "2.0"])
def test_oracle_pyarrow_files(enc, version):
    """pyarrow's writer and reader (independent of the generator and of the
    reference) agree with the oracle."""
    pa = pytest.importorskip("pyarrow")
    pq = pytest.importorskip("pyarrow.parquet")
    import pqgpu
    rng = np.random.default_rng(11)
    words = sorted("w%05d_%s" % (i, "xyz" * int(rng.integers(0, 9))) for i in range(2000))
    arr = pa.array([words[int(i)] if rng.random() > 0.1 else None for i in rng.integers(0, 2000, 9000)])
    buf = io.BytesIO()
    pq.write_table(pa.table({"s": arr}), buf, use_dictionary=False, column_encoding={"s": enc},
                   data_page_version=version, compression="snappy", data_page_size=20000)
    pf = pqgpu.ParquetFile(buf.getvalue())
    r = O.decode_chunk(pf.host_job(0, 0)[0])
    assert r.status == 0, abi.status_name(r.status)
    assert _strings(r) == [x.encode() for x in arr.to_pylist() if x is not None]


# ---------------------------------------------------------------- hand-built pages
def _dlba(lens, chars):
    return W.dbp_encode(np.asarray(lens, dtype=np.int32), bits=32) + bytes(chars)


def _dba(prefix, suffix_lens, chars):
    return W.dbp_encode(np.asarray(prefix, dtype=np.int32), bits=32) + _dlba(suffix_lens, chars)


def _huge_dlba(length, count, bad_width=False):
    """A DBP length stream announcing `count` lengths all equal to `length`:
    blocks of 2^30 values, 4 zero-width miniblocks each (a second block's
    widths > 32 with bad_width)."""
    bs = 1 << 30
    out = U.uvarint(bs) + U.uvarint(4) + U.uvarint(count) + U.zigzag(length)
    for b in range(-(-(count - 1) // bs)):
        out += U.uvarint(0) + bytes([40 if (bad_width and b == 1) else 0] * 4)
    return out


def _page_chunk(values_section, nvals, enc):
    return U.v1_page(values_section, nvals, enc)


def hand_cases():
    """(name, chunk bytes, expected oracle status) — statuses follow the cited lines."""
    ok_lens = [3, 0, 5, 2, 7, 1, 4, 4, 2]
    chars = bytes(range(97, 97 + sum(ok_lens)))
    n = len(ok_lens)
    cases = [
        ("dlba_ok", _page_chunk(_dlba(ok_lens, chars), n, DLBA), 0),
        # a negative length: make([]byte, size) panics in the reference -> BYTE_ARRAY
        ("dlba_negative", _page_chunk(_dlba([3, -2, 5, 2, 7, 1, 4, 4, 2], chars), n, DLBA),
         abi.STATUS_CODES["BYTE_ARRAY"]),
        # lengths past the page: io.ReadFull short -> EOF
        ("dlba_short", _page_chunk(_dlba(ok_lens, chars[:-3]), n, DLBA), abi.STATUS_CODES["EOF"]),
        # fewer lengths than values: next() at position >= len(lens) -> EOF
        ("dlba_few_lens", _page_chunk(_dlba(ok_lens[:5], chars[:sum(ok_lens[:5])]), n, DLBA),
         abi.STATUS_CODES["EOF"]),
        # Q3: one length, no miniblock header -> init fails (EOF)
        ("dlba_one_value", _page_chunk(_dlba([3], b"abc"), 1, DLBA), abi.STATUS_CODES["EOF"]),
        # more lengths than the page's values: every length is decoded (type_bytearray.go:104-113),
        # the value bytes start after all of them, the page takes its first 4 values
        ("dlba_more_lens", _page_chunk(_dlba(ok_lens, chars), 4, DLBA), 0),
        ("dba_more_lens", _page_chunk(_dba([0, 2, 2, 0, 1, 1, 0, 2, 2], ok_lens, chars), 5, DBA), 0),
        # ~2^31 zero-width lengths announced by two block headers: walked by block, not by value
        ("dlba_huge_count", _page_chunk(_huge_dlba(3, 2_000_000_000) + b"abcdefghi", 3, DLBA), 0),
        ("dlba_huge_count_bad_tail", _page_chunk(_huge_dlba(3, 2_000_000_000, bad_width=True) + b"abcdefghi", 3,
                                                 DLBA), abi.STATUS_CODES["BIT_WIDTH"]),
        ("dba_ok", _page_chunk(_dba([0, 2, 2, 0, 1, 1, 0, 2, 2], ok_lens, chars), n, DBA), 0),
        # prefix longer than the previous value -> "invalid prefix len in the stream"
        ("dba_prefix_too_long", _page_chunk(_dba([0, 2, 2, 0, 9, 1, 0, 2, 2], ok_lens, chars), n, DBA),
         abi.STATUS_CODES["BYTE_ARRAY"]),
        # different numbers of prefixes and suffixes
        ("dba_count_mismatch", _page_chunk(_dba([0, 2, 2, 0, 1, 1, 0, 2], ok_lens, chars), n, DBA),
         abi.STATUS_CODES["DELTA"]),
        # negative prefix + suffix capacity: panics in the reference -> BYTE_ARRAY
        ("dba_negative_capacity", _page_chunk(_dba([0, -9, 2, 0, 1, 1, 0, 2, 2], ok_lens, chars), n, DBA),
         abi.STATUS_CODES["BYTE_ARRAY"]),
        # a negative prefix with a long enough suffix is a plain suffix (no check fails)
        ("dba_negative_prefix", _page_chunk(_dba([0, 2, -1, 0, 1, 1, 0, 2, 2], ok_lens, chars), n, DBA), 0),
    ]
    return cases


@pytest.mark.parametrize("case", hand_cases(), ids=lambda c: c[0])
def test_oracle_hand_pages(case):
    name, chunk, want = case
    job, _ = U.chunk_job(chunk, ptype=abi.BYTE_ARRAY)
    r = O.decode_chunk(job)
    assert r.status == want, "%s: %s" % (name, abi.status_name(r.status))
    if name == "dlba_ok":
        assert b"".join(_strings(r)) == bytes(range(97, 97 + 28))
    if name == "dlba_more_lens":
        assert _strings(r) == [b"abc", b"", b"defgh", b"ij"]
    if name == "dlba_huge_count":
        assert _strings(r) == [b"abc", b"def", b"ghi"]
    if name == "dba_ok":
        got = _strings(r)
        assert len(got) == 9 and got[1][:2] == got[0][:2]


def flba_cases():
    """DELTA_BYTE_ARRAY on FIXED_LEN_BYTE_ARRAY (getFixedLenByteArrayValuesDecoder
    chunk_reader.go:90-91 -> byteArrayDeltaDecoder type_bytearray.go:189-240):
    (name, chunk, type_length, expected status).  Values of type_length bytes
    decode into the fixed-width output; a value of another length (which the
    reference would hand out as is) fails the page with FIXED_LEN."""
    # 9 values of 4 bytes: prefixes shared with the previous value
    pre = [0, 1, 1, 0, 4, 2, 0, 3, 3]
    suf = [4 - p for p in pre]
    chars = bytes(range(65, 65 + sum(suf)))
    bad_suf = list(suf)
    bad_suf[5] += 1
    return [
        ("flba_dba_ok", _page_chunk(_dba(pre, suf, chars), 9, DBA), 4, 0),
        ("flba_dba_len", _page_chunk(_dba(pre, bad_suf, chars + b"x"), 9, DBA), 4, abi.STATUS_CODES["FIXED_LEN"]),
        # the reference's own errors come first in value order
        ("flba_dba_prefix", _page_chunk(_dba([0, 1, 9, 0, 4, 2, 0, 3, 3], suf, chars), 9, DBA), 4,
         abi.STATUS_CODES["BYTE_ARRAY"]),
        ("flba_dba_tl0", _page_chunk(_dba(pre, bad_suf, chars + b"x"), 9, DBA), 0, 0),  # length 0: byte arrays
    ]


@pytest.mark.parametrize("case", flba_cases(), ids=lambda c: c[0])
def test_oracle_flba_delta_byte_array(case):
    name, chunk, tl, want = case
    job, _ = U.chunk_job(chunk, ptype=abi.FIXED_LEN_BYTE_ARRAY, type_length=tl)
    r = O.decode_chunk(job)
    assert r.status == want, "%s: %s" % (name, abi.status_name(r.status))
    if name == "flba_dba_ok":
        v = np.asarray(r.values).reshape(9, 4)
        assert bytes(v[1][:1]) == bytes(v[0][:1]) and bytes(v[4]) == bytes(v[3])


def test_oracle_flba_generated():
    """A generated FLBA(6) column written with DELTA_BYTE_ARRAY (prefixes
    shared with the previous value), nulls included: the oracle returns the
    generator's values, densely."""
    import pqgpu
    data, vals = _flba_file()
    pf = pqgpu.ParquetFile(data)
    r = O.decode_chunk(pf.host_job(0, 0)[0])
    assert r.status == 0, abi.status_name(r.status)
    assert r.value_width == 6 and np.array_equal(np.asarray(r.values), vals)


def _flba_file(rows=20000):
    rng = np.random.default_rng(21)
    defs = (rng.random(rows) >= 0.1).astype(np.uint8)
    nn = int(defs.sum())
    base = rng.integers(65, 91, size=(nn, 6)).astype(np.uint8)
    base[:, :3] = base[np.sort(rng.integers(0, nn, nn)), :3]  # shared prefixes
    vals = np.ascontiguousarray(base[np.lexsort(base.T[::-1])]).reshape(-1)
    col = W.Column("fx", W.FLBA, vals, type_length=6, repetition=W.OPTIONAL, def_levels=defs, encoding=DBA,
                   rows_per_page=3000)
    return W.write_file([col], rows), vals


# ---------------------------------------------------------------- GPU vs oracle
@pytest.fixture(scope="module")
def dec():
    import pqgpu
    d = pqgpu.GpuDecoder(0)
    yield d
    d.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kw", CASES, ids=lambda k: "e%d_v%d_c%d_n%d_s%d" % (
    k["encoding"], k["page_version"], k["codec"], int(k["null_frac"] * 100), k["sorted_values"]))
def test_gpu_generated_files(dec, kw):
    import pqgpu
    data, _ = W.config_delta_strings(rows=30000, rows_per_page=7000, **kw)
    pf = pqgpu.ParquetFile(data)
    dev = dec.upload(pf.data)
    try:
        r = dec.decode_jobs([pqgpu.device_job(pf, 0, 0, dev)])[0]
        P.compare_chunk(P.oracle_chunk(pf, 0, 0), dec.download(r, 0), "delta strings")
    finally:
        dec.free(dev)


@pytest.mark.gpu
def test_gpu_long_values_and_shared_prefixes(dec):
    """DELTA_BYTE_ARRAY values longer than the LDS buffers of k_str_dba (16 KiB
    previous value, 8 KiB suffix stage) and long shared prefixes."""
    rng = np.random.default_rng(12)
    base = bytes(rng.integers(97, 123, 40000, dtype=np.uint8))
    vals = sorted(base[:int(rng.integers(1, 40000))] + bytes([int(x)]) for x in rng.integers(97, 123, 300))
    vals += [b"z" * 20000, b"z" * 20001 + b"a", b"y"]
    offs = np.zeros(len(vals) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(v) for v in vals])
    chars = np.frombuffer(b"".join(vals), dtype=np.uint8).copy()
    for enc in (DBA, DLBA):
        col = W.Column("s", abi.BYTE_ARRAY, chars, offsets=offs, encoding=enc, rows_per_page=120)
        data = W.write_file([col], len(vals))
        import pqgpu
        pf = pqgpu.ParquetFile(data)
        exp = P.oracle_chunk(pf, 0, 0)
        assert exp.status == 0 and _strings(exp) == vals
        dev = dec.upload(pf.data)
        try:
            r = dec.decode_jobs([pqgpu.device_job(pf, 0, 0, dev)])[0]
            P.compare_chunk(exp, dec.download(r, 0), "long values enc %d" % enc)
        finally:
            dec.free(dev)


@pytest.mark.gpu
@pytest.mark.parametrize("case", hand_cases(), ids=lambda c: c[0])
def test_gpu_hand_pages(dec, case):
    P.compare_chunk_bytes(case[1], dec, ptype=abi.BYTE_ARRAY)


@pytest.mark.gpu
def test_gpu_mutations(dec):
    """Random byte flips in DLBA / DBA pages: the same status, error page and bytes as the oracle."""
    rng = np.random.default_rng(13)
    for enc in (DLBA, DBA):
        data, _ = W.config_delta_strings(rows=3000, rows_per_page=700, encoding=enc, codec=W.UNCOMPRESSED,
                                         null_frac=0.1)
        import pqgpu
        pf = pqgpu.ParquetFile(data)
        m = pf.chunk_meta(0, 0)
        chunk = bytes(pf.data[m.start:m.start + m.total_compressed_size])
        d = pf.columns[0].desc
        for _ in range(40):
            b = bytearray(chunk)
            for _ in range(int(rng.integers(1, 4))):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
            P.compare_chunk_bytes(bytes(b), dec, ptype=abi.BYTE_ARRAY, max_def=d.max_def)


@pytest.mark.gpu
@pytest.mark.parametrize("case", flba_cases(), ids=lambda c: c[0])
def test_gpu_flba_hand_pages(dec, case):
    P.compare_chunk_bytes(case[1], dec, ptype=abi.FIXED_LEN_BYTE_ARRAY, type_length=case[2])


@pytest.mark.gpu
def test_gpu_flba_generated(dec):
    data, _ = _flba_file()
    P.compare_file(data, dec)


def _odd_dbp(rng, n):
    """A DBP stream of n int32 values in an odd layout (block sizes not
    multiples of 128, miniblocks of 12 or 20 values, random widths)."""
    bs, mbc = [(12, 1), (40, 2), (24, 2), (128, 4), (64, 8)][int(rng.integers(0, 5))]
    mbvc = bs // mbc
    out = U.uvarint(bs) + U.uvarint(mbc) + U.uvarint(n) + U.zigzag(int(rng.integers(-50, 50)))
    vals = n - 1
    while vals > 0:
        widths = [int(rng.integers(0, 9)) for _ in range(mbc)]
        out += U.zigzag(int(rng.integers(-5, 5))) + bytes(widths)
        for w in widths:
            out += bytes(rng.integers(0, 256, (mbvc // 8) * w, dtype=np.uint8))
        vals -= bs
    return out


def test_oracle_dbp_skip_matches_next():
    """DeltaBP::skip_rest (lengths past NumValues) leaves the reader where
    next() for every value would, with the same status, on standard and odd
    layouts, truncated and mutated streams."""
    rng = np.random.default_rng(404)
    streams = []
    for _ in range(60):
        n = int(rng.integers(1, 3000))
        base = W.dbp_encode(rng.integers(0, 40, n).astype(np.int32), bits=32) if rng.random() < 0.5 \
            else _odd_dbp(rng, n)
        streams.append(base)
        streams.append(base[:int(rng.integers(1, len(base)))])
        b = bytearray(base)
        b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
        streams.append(bytes(b))
    checked = 0
    for s in streams:
        rc_full, end_full, cnt = O.delta_lengths_end(s, 1 << 40)
        if cnt > 200000:
            continue
        for keep in (0, 1, 5, 8, 9, 13, 64, 130, cnt // 2, max(cnt - 1, 0)):
            rc, end, _ = O.delta_lengths_end(s, keep)
            assert rc == rc_full, (keep, cnt, rc, rc_full)
            if rc == 0:  # (a failing stream fails the page: its reader position is not used)
                assert end == end_full, (keep, cnt, end, end_full)
            checked += 1
    assert checked > 1000
