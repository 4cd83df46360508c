"""Page-level, codec-level and ColumnStore-refill entries of the C ABI
(include/pqgpu.h): pqg_decode_page (pageReader.readValues), pqg_block_decompress
(BlockCompressor.DecompressBlock) and pqg_pack_levels (packedArray), each
against the oracle's counterpart, which the CPU tests pin to the reference's
own vectors."""
import ctypes as C
import json
import os

import numpy as np
import pytest

import parity as P
import pqtest_util as U
from gen import pqwrite as W
from oracle import pyoracle as O
from pqgpu import abi

GOLD = os.path.join(os.path.dirname(__file__), "golden")


# ---------------------------------------------------------------- CPU: oracle pinned to reference vectors
def test_oracle_pack_levels_matches_reference_kats():
    """packedArray's pack8 layout is the inverse of unpack8int32 (bitpacking32_test.go KATs)."""
    g = json.load(open(os.path.join(GOLD, "bitpack32.json")))
    n = 0
    for v in g["vectors"]:
        w = v["width"]
        if w == 0 or w > 8 or max(v["values"]) > 255:
            continue
        got = O.pack_levels(np.array(v["values"], np.uint8), (1 << w) - 1)
        assert got.tobytes() == bytes.fromhex(v["data"]), v
        n += 1
    assert n > 20


def test_oracle_pack_levels_roundtrip():
    rng = np.random.default_rng(1)
    for maxl in (1, 2, 3, 7, 200):
        lv = rng.integers(0, maxl + 1, size=1003).astype(np.uint8)
        packed = O.pack_levels(lv, maxl)
        bw = maxl.bit_length()
        assert len(packed) == (len(lv) + 7) // 8 * bw
        bits = np.unpackbits(packed, bitorder="little").reshape(-1, bw)
        back = (bits * (1 << np.arange(bw))).sum(axis=1)[: len(lv)]
        assert np.array_equal(back, lv)


# ---------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def dec():
    import pqgpu
    d = pqgpu.GpuDecoder(0)
    yield d
    d.close()


def _page_parts(chunk_bytes, ptype, **kw):
    """Split a hand-built chunk into (dict page bytes or b'', [data page bytes]) by walking headers with the oracle."""
    job, buf = U.chunk_job(chunk_bytes, ptype=ptype, **kw)
    ch = O.decode_chunk(job)
    pages = list(ch.pages)
    bounds = [p.header_offset for p in pages] + [len(chunk_bytes)]
    parts = [(pages[i].page_type, chunk_bytes[bounds[i]:bounds[i + 1]]) for i in range(len(pages))]
    d = b"".join(b for t, b in parts if t == abi.PAGE_DICTIONARY)
    return d, [b for t, b in parts if t != abi.PAGE_DICTIONARY]


def _decode_page(dec, col, page, dict_page=b""):
    pj = abi.PageJob()
    pj.col = col
    pp = dec.upload(page)
    dp = dec.upload(dict_page) if dict_page else None
    pj.page, pj.page_len = pp, len(page)
    pj.dict_page, pj.dict_page_len = dp, len(dict_page)
    r = abi.ChunkResult()
    rc = dec.L.pqg_decode_page(dec.ctx, C.byref(pj), C.byref(r))
    assert rc == 0, rc
    got = dec.download(r, 0)
    for p in (pp, dp):
        if p:
            dec.free(p)
    return got


@pytest.mark.gpu
def test_decode_page_matches_oracle_page_by_page(dec):
    """Every data page of multi-page chunks (dictionary pages, nulls, lists,
    strings, V2, snappy) decoded on its own equals the oracle's decode of that
    page behind the same dictionary."""
    import pqgpu
    rng = np.random.default_rng(4)
    cases = [W.config_c2(rows=9000, bits=7, rows_per_page=2500)[0],
             W.config_c4(rows=6000, vocab=900, rows_per_page=1500, dict_limit=6000)[0],
             W.config_c5(row_groups=(1,), rows_per_rg=5000, rows_per_page=1700)[0],
             W.config_c3(rows=7000, rows_per_page=3000)[0]]
    n = 0
    for data in cases:
        pf = pqgpu.ParquetFile(data)
        for c in range(pf.num_columns):
            m = pf.chunk_meta(0, c)
            chunk = pf.data[m.start:m.start + m.total_compressed_size]
            desc = pf.columns[c].desc
            dsc = abi.ColumnDesc()
            C.memmove(C.byref(dsc), C.byref(desc), C.sizeof(dsc))
            dsc.codec = m.codec
            kw = dict(max_def=desc.max_def, max_rep=desc.max_rep, codec=m.codec, type_length=desc.type_length)
            dict_page, pages = _page_parts(chunk, desc.physical_type, **kw)
            for page in pages:
                exp_job, _ = U.chunk_job(dict_page + page, ptype=desc.physical_type, **kw)
                exp = O.decode_chunk(exp_job)
                got = _decode_page(dec, dsc, page, dict_page)
                P.compare_chunk(exp, got, "col%d page" % c)
                n += 1
    assert n > 30


@pytest.mark.gpu
def test_block_decompress_matches_snappy_decode(dec):
    rng = np.random.default_rng(6)
    blocks = [b"", b"a", bytes(rng.integers(0, 256, 5000, dtype=np.uint8)), b"abcd" * 20000,
              bytes(rng.integers(0, 4, 200_000, dtype=np.uint8)), bytes(70_000)]
    comp = [W.snappy_compress(b) for b in blocks]
    bad = [comp[3][:-3], b"\xff\xff\xff\xff\xff\x01", comp[2][:1] + b"\x0e\xff\xff",
           W.snappy_compress(b"xyz" * 50)[:-1] + b"\x33"]
    for src in comp + bad:
        rc_o, out_o = O.snappy_decode(src)
        cap = 1 << 21
        dst = np.zeros(cap, np.uint8)
        n = C.c_int64(0)
        rc = dec.L.pqg_block_decompress(dec.ctx, abi.CODEC_SNAPPY, src, len(src), dst.ctypes.data, cap, C.byref(n))
        # same status class as snappy.Decode's restatement (ErrCorrupt -> SNAPPY)
        assert rc == rc_o, (rc, rc_o)
        if rc_o == 0:
            assert dst[:n.value].tobytes() == out_o
    # too small an output buffer; uncompressed copies; GZIP
    n = C.c_int64(0)
    dst = np.zeros(10, np.uint8)
    assert dec.L.pqg_block_decompress(dec.ctx, abi.CODEC_SNAPPY, comp[2], len(comp[2]), dst.ctypes.data, 10,
                                      C.byref(n)) == abi.ERR_CAPACITY and n.value == 5000
    assert dec.L.pqg_block_decompress(dec.ctx, abi.CODEC_UNCOMPRESSED, b"12345", 5, dst.ctypes.data, 10,
                                      C.byref(n)) == 0 and dst[:5].tobytes() == b"12345"
    assert dec.L.pqg_block_decompress(dec.ctx, abi.CODEC_GZIP, b"12345", 5, dst.ctypes.data, 10,
                                      C.byref(n)) == abi.STATUS_CODES["GZIP"]  # not a gzip member


@pytest.mark.gpu
@pytest.mark.parametrize("maxl", [1, 2, 3, 7, 255])
def test_pack_levels_matches_oracle(dec, maxl):
    rng = np.random.default_rng(maxl)
    for n in (0, 1, 7, 8, 9, 1000, 123457):
        lv = rng.integers(0, maxl + 1, size=n).astype(np.uint8)
        exp = O.pack_levels(lv, maxl)
        lp = dec.upload(lv) if n else None
        out_n = max(len(exp), 1)
        op = dec.upload(np.zeros(out_n, np.uint8))
        assert dec.L.pqg_pack_levels(dec.ctx, lp, n, maxl, op) == 0
        assert np.array_equal(dec.d2h(op, len(exp)), exp)
        for p in (lp, op):
            if p:
                dec.free(p)


@pytest.mark.gpu
def test_product_rejects_quirks(dec):
    job, buf = U.chunk_job(U.v1_page(np.array([1], np.int32).tobytes(), 1, 0), ptype=abi.INT32)
    dev = dec.upload(buf)
    job.data = dev
    job.quirks = abi.QUIRK_Q1_PAGE_NILS
    res = (abi.ChunkResult * 1)()
    assert dec.L.pqg_decode_chunks(dec.ctx, C.byref(job), 1, res) == abi.STATUS_CODES["INVALID_ARG"]
    dec.free(dev)


@pytest.mark.gpu
def test_unsigned_flag_reaches_result(dec):
    """The unsigned bit of pqg_column_desc.flags (set by the planner from the
    schema, chunk_reader.go:99-141) comes back in pqg_chunk_result.col_flags, so
    the Go adapter boxes uint32/uint64 like int32PlainDecoder.unSigned
    (type_int32.go:29-33); the value bits are the same either way."""
    import pqgpu
    data = open(os.path.join(GOLD, "unsigned.parquet"), "rb").read()
    pf = pqgpu.ParquetFile(data)
    dev = dec.upload(pf.data)
    try:
        for c in range(pf.num_columns):
            exp = O.decode_chunk(pf.host_job(0, c)[0])
            outs = []
            for flags in (pf.columns[c].desc.flags, pf.columns[c].desc.flags ^ 1):
                job = pqgpu.device_job(pf, 0, c, dev)
                job.col.flags = flags
                r = dec.decode_jobs([job])[0]
                assert r.col_flags == flags
                outs.append(dec.download(r, 0))
                P.compare_chunk(exp, outs[-1], "unsigned col %d flags %d" % (c, flags))
            assert outs[0].values.tobytes() == outs[1].values.tobytes()
    finally:
        dec.free(dev)


@pytest.mark.gpu
def test_file_reader_projection_uploads_selected_span(tmp_path):
    """pqgpu.FileReader (NewFileReader(r, columns...) file_reader.go:27-48,
    isSelected schema.go:296-312): a path-backed reader uploads only the selected
    chunks' byte span per row group and decodes them like the oracle."""
    import pqgpu
    data, _ = W.config_c5(row_groups=(0, 1), rows_per_rg=6000, rows_per_page=2000)
    path = tmp_path / "c5.parquet"
    path.write_bytes(data)
    pf = pqgpu.ParquetFile(data)
    dec = pqgpu.GpuDecoder(0)
    try:
        fr = pqgpu.FileReader(str(path), "i64d", "s", decoder=dec)
        sel = [pf.column_index("i64d"), pf.column_index("s")]
        assert fr.selected == sel
        for rg in range(2):
            got = fr.read_row_group(rg)
            assert sorted(got) == ["i64d", "s"]
            for c in sel:
                P.compare_chunk(P.oracle_chunk(pf, rg, c), got[pf.columns[c].path.decode()], "rg%d col%d" % (rg, c))
        ranges = [pqgpu.chunk_ranges(pf, [(rg, c) for c in sel])[0] for rg in range(2)]
        want = sum(hi - lo for rs in ranges for lo, hi in rs)
        metas = [pf.chunk_meta(rg, c) for rg in range(2) for c in sel]
        assert fr.uploaded_bytes == want == sum(m.total_compressed_size for m in metas) < len(data) // 2
        lst = pqgpu.FileReader(str(path), "lst", decoder=dec)  # a group prefix selects its leaves
        assert [pf.columns[c].path.decode() for c in lst.selected] == ["lst.list.element"]
    finally:
        dec.close()
