"""GPU parity: libpqgpu (HIP, gfx950) vs the CPU oracle, bit-exact, through the C ABI.

Sizes here are small enough for the oracle to finish in seconds; the
full-size configs are checked by bench.py's verify pass against the
generator's own arrays (`verified_bit_exact`), and cases larger than the
kernels' LDS windows (long runs, >= 1 MiB snappy pages, long DBA values) by
test_levels.py, test_snappy_split.py and test_delta_strings.py.
"""
import json
import os

import numpy as np
import pytest

import parity as P
import pqtest_util as U
from gen import pqwrite as W
from pqgpu import abi

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def dec():
    import pqgpu
    d = pqgpu.GpuDecoder(0)
    yield d
    d.close()


@pytest.fixture(scope="module")
def dec_scan():
    """A decoder without the K1 stride walk (PQG_STRIDE=0, read at context
    creation): chunks of equal pages then take the candidate scan, which the
    scan tests below exercise."""
    import os
    import pqgpu
    old = os.environ.get("PQG_STRIDE")
    os.environ["PQG_STRIDE"] = "0"
    try:
        d = pqgpu.GpuDecoder(0)
    finally:
        if old is None:
            os.environ.pop("PQG_STRIDE", None)
        else:
            os.environ["PQG_STRIDE"] = old
    yield d
    d.close()


def test_c1_plain_int64(dec):
    data, _ = W.config_c1(rows=200_000, rows_per_page=20000)
    P.compare_file(data, dec)
    data, _ = W.config_c1(rows=100_003, rows_per_page=100_003)  # 1-page variant
    P.compare_file(data, dec)


@pytest.mark.parametrize("bits", [0, 1, 2, 4, 8, 12, 16, 20])
def test_c2_dict_uniform(dec, bits):
    data, _ = W.config_c2(rows=60_000, bits=bits, rows_per_page=20000)
    P.compare_file(data, dec)


@pytest.mark.parametrize("bits", [1, 8, 20])
def test_c2_dict_run_heavy(dec, bits):
    data, _ = W.config_c2(rows=60_000, bits=bits, run_heavy=True, rows_per_page=7000)
    P.compare_file(data, dec)


def test_c2_v2_snappy(dec):
    data, _ = W.config_c2(rows=50_000, bits=8, page_version=2, codec=W.SNAPPY, rows_per_page=6000)
    P.compare_file(data, dec)


def test_c2_v1_snappy(dec):
    data, _ = W.config_c2(rows=50_000, bits=12, page_version=1, codec=W.SNAPPY, rows_per_page=6000)
    P.compare_file(data, dec)


def test_c3_delta_v2_snappy(dec):
    data, _ = W.config_c3(rows=100_000, rows_per_page=20000)
    P.compare_file(data, dec)


def test_c3_delta_uncompressed_large_page(dec):
    data, _ = W.config_c3(rows=50_001, rows_per_page=50_001, codec=W.UNCOMPRESSED)
    P.compare_file(data, dec)


def test_delta_int32_and_widths(dec):
    rng = np.random.default_rng(3)
    for n in (2, 9, 130, 1000, 20000):
        v = rng.integers(-2**31, 2**31 - 1, size=n, dtype=np.int64).astype(np.int32)
        data = W.write_file([W.Column("d", W.INT32, v, encoding=W.DELTA_BINARY_PACKED, rows_per_page=n)], n)
        P.compare_file(data, dec)
        w = rng.integers(-2**63, 2**63 - 1, size=n, dtype=np.int64)
        data = W.write_file([W.Column("d", W.INT64, w, encoding=W.DELTA_BINARY_PACKED, rows_per_page=n)], n)
        P.compare_file(data, dec)


def test_delta_q3_errors_match(dec):
    for n in (1, 129, 257):
        v = np.arange(n, dtype=np.int64) * 7
        data = W.write_file([W.Column("d", W.INT64, v, encoding=W.DELTA_BINARY_PACKED, rows_per_page=n)], n)
        res = P.compare_file(data, dec)
        assert res[0].status == -1  # EOF, like the oracle (Q3)


def test_plain_types(dec):
    rng = np.random.default_rng(5)
    n = 12_345
    f32 = rng.standard_normal(n).astype(np.float32)
    f32[::97] = np.nan
    f32.view(np.uint32)[::101] = 0x7FC00001  # NaN payloads survive bit-exact
    cols = [W.Column("f", W.FLOAT, f32, rows_per_page=1000),
            W.Column("d", W.DOUBLE, rng.standard_normal(n), rows_per_page=999),
            W.Column("b", W.BOOLEAN, rng.integers(0, 2, n).astype(np.uint8), rows_per_page=1001),
            W.Column("fx", W.FLBA, rng.integers(0, 256, size=n * 5, dtype=np.uint8), type_length=5,
                     rows_per_page=700),
            W.Column("i96", W.INT96, rng.integers(0, 256, size=n * 12, dtype=np.uint8), rows_per_page=333),
            W.Column("i32", W.INT32, rng.integers(-2**31, 2**31 - 1, n).astype(np.int32), rows_per_page=4096),
            W.Column("o64", W.INT64, rng.integers(0, 10, n - 100), repetition=W.OPTIONAL,
                     def_levels=np.r_[np.ones(n - 100), np.zeros(100)][rng.permutation(n)].astype(np.uint8),
                     rows_per_page=3000, codec=W.SNAPPY, page_version=2)]
    data = W.write_file(cols, n, row_groups=2)
    P.compare_file(data, dec)


def test_dict_other_types(dec):
    rng = np.random.default_rng(8)
    n = 20000
    cols = [W.Column("dd", W.DOUBLE, rng.integers(0, 50, n).astype(np.float64), encoding=W.RLE_DICTIONARY),
            W.Column("di", W.INT64, rng.integers(0, 300, n), encoding=W.RLE_DICTIONARY, codec=W.SNAPPY),
            W.Column("dfx", W.FLBA, np.repeat(rng.integers(0, 256, size=(40, 3), dtype=np.uint8), n // 40, axis=0),
                     type_length=3, encoding=W.RLE_DICTIONARY),
            W.Column("d96", W.INT96, np.tile(rng.integers(0, 256, size=12 * 7, dtype=np.uint8), n // 7 + 1)[: n * 12],
                     encoding=W.RLE_DICTIONARY, page_version=2)]
    data = W.write_file(cols, n)
    P.compare_file(data, dec)


def test_list_levels(dec):
    rng = np.random.default_rng(9)
    rows = 20000
    lens = rng.integers(0, 4, size=rows)
    rep, defs, vals = [], [], []
    for r in range(rows):
        if rng.random() < 0.05:
            rep.append(0); defs.append(0)
        elif lens[r] == 0:
            rep.append(0); defs.append(1)
        else:
            for k in range(lens[r]):
                rep.append(0 if k == 0 else 1)
                if rng.random() < 0.05:
                    defs.append(2)
                else:
                    defs.append(3); vals.append(rng.standard_normal())
    for pv in (1, 2):
        col = W.Column("l", W.DOUBLE, np.array(vals), repetition=W.LIST, def_levels=np.array(defs),
                       rep_levels=np.array(rep), rows_per_page=2500, page_version=pv)
        data = W.write_file([col], rows, row_groups=2)
        P.compare_file(data, dec)


def test_dremel_twitter_levels(dec):
    g = json.load(open(os.path.join(GOLD, "dremel.json")))
    rep = W.hybrid_encode(g["rep_levels"], 2)
    defs = W.hybrid_encode(g["def_levels"], 2)
    vals = np.array(g["values"], dtype=np.int32).tobytes()
    page = U.v1_page(vals, len(g["rep_levels"]), 0, rep=rep, defs=defs)
    exp, got = P.compare_chunk_bytes(page, dec, ptype=abi.INT32, max_def=2, max_rep=2)
    assert got.rep_levels.tolist() == g["rep_levels"]


def _hand_cases():
    """Hand-built chunks covering the reference's error paths and quirks."""
    H = W.hybrid_encode
    cases = []
    i32 = lambda a: np.array(a, dtype=np.int32).tobytes()  # noqa: E731
    # dictionary chunk, valid
    dpage = U.page_header_dict(16, 16, 4) + i32([10, 20, 30, 40])
    idx = bytes([2]) + H([0, 1, 2, 3, 3, 2, 1, 0, 1], 2)
    cases.append(("dict_ok", dpage + U.v1_page(idx, 9, 8), dict(ptype=abi.INT32)))
    # dict index out of range
    idx = bytes([3]) + H([0, 1, 7], 3)
    cases.append(("dict_bad_index", dpage + U.v1_page(idx, 3, 8), dict(ptype=abi.INT32)))
    # dict width byte > 32
    cases.append(("dict_bad_width", dpage + U.v1_page(bytes([33]), 3, 8), dict(ptype=abi.INT32)))
    # dict without a dictionary page
    cases.append(("dict_missing", U.v1_page(bytes([2]) + H([0, 1], 2), 2, 8), dict(ptype=abi.INT32)))
    # second dictionary page
    cases.append(("two_dicts", dpage + dpage + U.v1_page(bytes([2]) + H([0], 2), 1, 8), dict(ptype=abi.INT32)))
    # empty values section of a dict page with all-null levels (init still reads the width byte)
    cases.append(("dict_all_null_no_width", dpage + U.v1_page(b"", 3, 8, defs=H([0, 0, 0], 1)),
                  dict(ptype=abi.INT32, max_def=1)))
    # PLAIN truncated
    cases.append(("plain_short", U.v1_page(i32([1, 2, 3])[:-1], 3, 0), dict(ptype=abi.INT32)))
    # trailing bytes ignored (Q7)
    cases.append(("plain_trailing", U.v1_page(i32([1, 2, 3]) + b"xyz", 3, 0), dict(ptype=abi.INT32)))
    # hybrid: empty runs, oversized RLE value, exhausted stream
    cases.append(("levels_empty_bp", U.v1_page(i32([1]), 1, 0, defs=b"\x01"), dict(ptype=abi.INT32, max_def=1)))
    cases.append(("levels_empty_rle", U.v1_page(i32([1]), 1, 0, defs=b"\x00\x01"), dict(ptype=abi.INT32, max_def=1)))
    cases.append(("levels_big_rle", U.v1_page(i32([1]), 1, 0, defs=b"\x02\x02"), dict(ptype=abi.INT32, max_def=1)))
    cases.append(("levels_short", U.v1_page(i32([1, 2]), 5, 0, defs=b"\x04\x01"), dict(ptype=abi.INT32, max_def=1)))
    # run headers as long varints (binary.ReadUvarint accepts zero high bytes up to 10 bytes)
    one = dict(ptype=abi.INT32, max_def=1)
    cases.append(("levels_varint6", U.v1_page(i32([1]), 1, 0, defs=b"\x82\x80\x80\x80\x80\x00\x01"), one))
    cases.append(("levels_varint10", U.v1_page(i32([1]), 1, 0, defs=b"\x82" + b"\x80" * 8 + b"\x00\x01"), one))
    cases.append(("levels_varint11", U.v1_page(i32([1]), 1, 0, defs=b"\x82" + b"\x80" * 9 + b"\x00\x01"), one))
    cases.append(("levels_varint_gt_int32", U.v1_page(i32([1]), 1, 0, defs=b"\x80\x80\x80\x80\x10\x01"), one))
    cases.append(("levels_varint_eof", U.v1_page(i32([1]), 1, 0, defs=b"\x80"), one))
    cases.append(("levels_bp_2byte_header",
                  U.v1_page(i32(list(range(800))), 800, 0, defs=b"\xc9\x01" + b"\xff" * 100), one))
    # Q5: short bit-packed group zero padded
    cases.append(("levels_q5", U.v1_page(i32([7]), 3, 0, defs=b"\x03\x01"), dict(ptype=abi.INT32, max_def=1)))
    # V1 level length prefix missing
    cases.append(("levels_no_prefix", U.page_header_v1(2, 2, 1, 0) + b"\x01\x00", dict(ptype=abi.INT32, max_def=1)))
    # level encoding not RLE
    cases.append(("levels_bitpacked_enc", U.page_header_v1(4, 4, 1, 0, def_enc=4) + i32([1]),
                  dict(ptype=abi.INT32, max_def=1)))
    # unsupported value encoding
    cases.append(("enc_unsupported", U.v1_page(i32([1]), 1, 6), dict(ptype=abi.INT32)))
    # V2 with zero-length def levels but max_def > 0: reader not initialised
    body = i32([5])
    cases.append(("v2_no_levels", U.page_header_v2(4, 4, 1, 0, 1, 0, 0, 0) + body, dict(ptype=abi.INT32, max_def=1)))
    # V2 is_compressed=false + SNAPPY codec: the reference ignores the flag (Q4)
    raw = i32([1, 2, 3])
    cases.append(("v2_q4", U.page_header_v2(12, 12, 3, 0, 3, 0, 0, 0, is_comp=False) + raw,
                  dict(ptype=abi.INT32, codec=1)))
    # snappy corrupt / size mismatch
    comp = W.snappy_compress(raw)
    cases.append(("snappy_ok", U.page_header_v1(12, len(comp), 3, 0) + comp, dict(ptype=abi.INT32, codec=1)))
    cases.append(("snappy_size", U.page_header_v1(13, len(comp), 3, 0) + comp, dict(ptype=abi.INT32, codec=1)))
    bad = comp[:-2] + b"\x09\x00"
    cases.append(("snappy_corrupt", U.page_header_v1(12, len(bad), 3, 0) + bad, dict(ptype=abi.INT32, codec=1)))
    # uncompressed size mismatch
    cases.append(("uncomp_size", U.page_header_v1(13, 12, 3, 0) + raw, dict(ptype=abi.INT32)))
    # page body shorter than compressed size
    cases.append(("short_body", U.page_header_v1(40, 40, 3, 0) + raw, dict(ptype=abi.INT32)))
    # index page type / garbage header
    t = U.TW()
    t.i32(1, 1).i32(2, 0).i32(3, 0)
    cases.append(("index_page", t.stop(), dict(ptype=abi.INT32)))
    cases.append(("garbage_header", b"\x15\x00\x15", dict(ptype=abi.INT32)))
    cases.append(("negative_values", U.page_header_v1(0, 0, -1, 0), dict(ptype=abi.INT32)))
    # header with unknown fields / nested structs / maps to skip
    t = U.TW()
    t.i32(1, 0).i32(2, 4).i32(3, 4)
    t.begin(5).i32(1, 1).i32(2, 0).i32(3, 3).i32(4, 3).end()
    t.i64(12, 77)
    t.b += bytes([0x1b, 0x01, 0x55, 0x02, 0x04])  # field 13 map<i32,i32> {1: 2}
    t.last[-1] = 13
    cases.append(("skip_fields", t.stop() + i32([9]), dict(ptype=abi.INT32)))
    # a header whose unknown field is a LIST<STRUCT> of 2^30 elements at the end of
    # the bytes: every element is an empty struct at EOF (skipped at once, not
    # 2^30 times), then the header fails like the reference's
    t = U.TW()
    t.i32(1, 0).i32(2, 4).i32(3, 4)
    cases.append(("huge_struct_list", t.b + bytes([0xA9, 0xFC]) + U.uvarint(1 << 30), dict(ptype=abi.INT32)))
    t = U.TW()
    t.i32(1, 0).i32(2, 4).i32(3, 4)
    cases.append(("huge_struct_map", t.b + bytes([0xAB]) + U.uvarint(1 << 30) + bytes([0xC5]),
                  dict(ptype=abi.INT32)))
    # INT96 truncated final value: left nil (Q8)
    cases.append(("int96_q8", U.v1_page(bytes(range(30)), 3, 0), dict(ptype=abi.INT96)))
    cases.append(("int96_short", U.v1_page(bytes(range(24)), 3, 0), dict(ptype=abi.INT96)))
    # boolean RLE
    cases.append(("bool_rle", U.v1_page(U.u32(len(H([1, 0, 1, 1], 1))) + H([1, 0, 1, 1], 1), 4, 3),
                  dict(ptype=abi.BOOLEAN)))
    # delta: invalid block size / miniblock count / bit width
    cases.append(("delta_bad_mb", U.v1_page(bytes([0x80, 0x01, 0x03, 0x05, 0x00]), 5, 5), dict(ptype=abi.INT64)))
    cases.append(("delta_bad_width", U.v1_page(bytes([0x80, 0x01, 0x04, 0x05, 0x00, 0x00, 65, 0, 0, 0]), 5, 5),
                  dict(ptype=abi.INT64)))
    cases.append(("delta_zero_block", U.v1_page(bytes([0x00, 0x01, 0x05, 0x00]), 5, 5), dict(ptype=abi.INT64)))
    # delta with an odd miniblock layout (block 12, 1 miniblock): generic path
    dv = bytes([12, 1, 20, 0]) + bytes([0, 3]) + bytes(range(3)) * 2 + bytes([0, 3]) + bytes(range(9))
    cases.append(("delta_odd_layout", U.v1_page(dv, 20, 5), dict(ptype=abi.INT32)))
    dv = bytes([20, 1, 12, 10]) + bytes([2, 4]) + bytes([0x21, 0x43, 0x65, 0x87, 0xa9, 0xcb, 0xed, 0x0f])
    cases.append(("delta_odd_ok", U.v1_page(dv, 12, 5), dict(ptype=abi.INT32)))
    cases.append(("delta_odd_ok64", U.v1_page(dv, 12, 5), dict(ptype=abi.INT64)))
    return cases


@pytest.mark.parametrize("case", _hand_cases(), ids=lambda c: c[0])
def test_hand_built(dec, case):
    name, chunk, kw = case
    P.compare_chunk_bytes(chunk, dec, **kw)


def test_crash_files(dec):
    import pqgpu
    files = json.load(open(os.path.join(GOLD, "crash_files.json")))["files"]
    for f in files:
        data = bytes.fromhex(f["data"])
        try:
            pf = pqgpu.ParquetFile(data)
        except pqgpu.PqgError:
            continue
        ok_cols = []
        for c in range(pf.num_columns):
            try:
                for rg in range(pf.num_row_groups):
                    pf.chunk_meta(rg, c)
                ok_cols.append(c)
            except pqgpu.PqgError:
                pass
        if ok_cols:
            P.compare_file(data, dec, cols=ok_cols)


def test_fuzz_mutations(dec):
    """Random byte flips of small valid files: GPU and oracle agree on status and bytes."""
    import pqgpu
    rng = np.random.default_rng(1234)
    bases = [W.config_c2(rows=3000, bits=5, rows_per_page=700)[0],
             W.config_c3(rows=2000, rows_per_page=600)[0],
             W.config_c1(rows=2000, rows_per_page=500)[0],
             W.config_c2(rows=2000, bits=3, rows_per_page=600, page_version=2, codec=W.SNAPPY)[0]]
    n_cases = 0
    for base in bases:
        pf = pqgpu.ParquetFile(base)
        m = pf.chunk_meta(0, 0)
        lo, hi = m.start, m.start + m.total_compressed_size
        for _ in range(60):
            b = bytearray(base)
            for _ in range(int(rng.integers(1, 4))):
                pos = int(rng.integers(lo, hi))
                b[pos] = int(rng.integers(0, 256))
            P.compare_file(bytes(b), dec)
            n_cases += 1
    assert n_cases == 240


def _decode_one(dec, data):
    """Decode every chunk of `data` on the GPU, compare with the oracle, and
    return the K1 diagnostics of job 0 (serial_walk, candidates, pages, scratch)."""
    P.compare_file(data, dec)
    return dec.debug_job(0)[:4]


def test_scan_speculative_path_used(dec):
    # ordinary multi-page chunks: the parallel candidate scan settles the page list
    data, _ = W.config_c2(rows=200_000, bits=8, rows_per_page=20000)
    walk, cands, pages, _ = _decode_one(dec, data)
    assert walk == 0 and pages == 11 and cands >= pages
    data, _ = W.config_c3(rows=100_000, rows_per_page=20000)
    walk, cands, pages, scratch = _decode_one(dec, data)
    assert walk == 0 and pages == 5 and scratch > 0


def test_scan_big_pages_prewalked(dec):
    # a chunk of <= 4 big pages (parquet-go's writer: one page per chunk) is
    # walked before the candidate scan (serial_walk == 2) and skipped by it
    data, _ = W.config_c1(rows=100_003, rows_per_page=100_003)
    walk, cands, pages, _ = _decode_one(dec, data)
    assert walk == 2 and pages == 1 and cands == 0
    data = W.config_c4(rows=40_000, vocab=3000, rows_per_page=40_000, codec=W.UNCOMPRESSED)[0]
    walk, _, pages, _ = _decode_one(dec, data)
    assert walk == 2 and pages == 2  # dictionary page + one data page
    data, _ = W.config_c1(rows=40_000, rows_per_page=10_000)  # 4 pages of 1/4: walked
    walk, _, pages, _ = _decode_one(dec, data)
    assert walk == 2 and pages == 4
    # an understated TotalCompressedSize / a damaged big page: still the oracle's result
    data, _ = W.config_c1(rows=100_003, rows_per_page=100_003)
    b = bytearray(data)
    b[6] ^= 0xFF
    P.compare_file(bytes(b), dec)


def test_scan_false_candidates_are_skipped(dec_scan):
    # PLAIN int32 payload bytes 15 00 15 00 parse as page-header prefixes: a few
    # per tile are false candidates the chain must jump over
    n = 60_000
    v = np.arange(n, dtype=np.int32)
    v[::997] = 0x00150015
    data = W.write_file([W.Column("x", W.INT32, v, rows_per_page=5000)], n)
    walk, cands, pages, _ = _decode_one(dec_scan, data)
    assert walk == 0 and pages == 12 and cands > pages


def test_scan_false_ok_headers_walked(dec_scan):
    # a complete, valid DataPageHeader embedded in PLAIN payload bytes: an ok
    # false candidate between two real pages (the chain is walked around it)
    fake = bytes([0x15, 0x00, 0x15, 0x02, 0x15, 0x02, 0x2C, 0x15, 0x02, 0x15, 0x00, 0x15, 0x00, 0x15, 0x00,
                  0x00, 0x00, 0, 0, 0])
    n = 60_000
    v = np.arange(n, dtype=np.int32)
    fk = np.frombuffer(fake, dtype=np.int32)
    for at in range(1000, n - 10, 7919):
        v[at:at + len(fk)] = fk
    for codec in (W.UNCOMPRESSED, W.SNAPPY):
        data = W.write_file([W.Column("x", W.INT32, v, rows_per_page=5000, codec=codec)], n)
        walk, cands, pages, _ = _decode_one(dec_scan, data)
        assert walk == 0 and pages == 12


def test_scan_stride_walk(dec):
    # equal pages (fixed-width PLAIN, rows per page fixed): the prewalk checks
    # the predicted page positions 64 at a time and the candidate scan is skipped
    n = 200_003
    v = np.arange(n, dtype=np.int64) * 7
    data = W.write_file([W.Column("x", W.INT64, v, rows_per_page=1000)], n)  # 201 pages, the last short
    walk, cands, pages, _ = _decode_one(dec, data)
    assert walk == 2 and cands == 0 and pages == 201
    # a dictionary page first, then equal data pages (the serial part, then the stride)
    data = W.config_c4(rows=30_000, vocab=500, rows_per_page=1000, codec=W.UNCOMPRESSED)[0]
    P.compare_file(data, dec)
    # optional columns: equal pages only when the null pattern is regular
    d = (np.arange(n) % 3 != 0).astype(np.uint8)
    vv = v[d.astype(bool)]
    data = W.write_file([W.Column("x", W.INT64, vv, repetition=W.OPTIONAL, def_levels=d, rows_per_page=999)], n)
    P.compare_file(data, dec)


def test_scan_stride_walk_mispredicted(dec):
    # damaged headers at predicted page positions, a page of another length,
    # bytes past the last page: the stride walk gives up (or reads the same
    # error) and the result is the oracle's
    import pqgpu
    n = 60_000
    v = np.arange(n, dtype=np.int32)
    data = W.write_file([W.Column("x", W.INT32, v, rows_per_page=5000)], n)
    m = pqgpu.ParquetFile(data).chunk_meta(0, 0)
    L = data.index(b"\x15\x00\x15", m.start + 3) - m.start  # the first page's length
    rng = np.random.default_rng(41)
    for _ in range(16):
        b = bytearray(data)
        k = int(rng.integers(1, n // 5000))
        b[m.start + k * L + int(rng.integers(0, 12))] ^= int(rng.integers(1, 256))
        P.compare_file(bytes(b), dec)
    # one page of another length in the middle
    v2 = np.concatenate([v[:20000], v[:1], v[20000:]])
    cols = [W.Column("x", W.INT32, v2, rows_per_page=5000)]
    P.compare_file(W.write_file(cols, n + 1), dec)


def test_scan_tile_overflow_falls_back(dec_scan):
    # every value is a header prefix: > kCandPerTile hits per tile -> serial walk
    n = 40_000
    v = np.full(n, 0x00150015, dtype=np.int32)
    data = W.write_file([W.Column("x", W.INT32, v, rows_per_page=9000)], n)
    walk, _, pages, _ = _decode_one(dec_scan, data)
    assert walk == 1 and pages == 5


def test_scan_tiny_pages(dec, dec_scan):
    # many pages per 16 KiB tile (fallback or not, the page list must match);
    # with the stride walk too (715 equal pages of ~90 bytes)
    n = 5000
    v = np.arange(n, dtype=np.int64)
    data = W.write_file([W.Column("x", W.INT64, v, rows_per_page=7)], n)
    P.compare_file(data, dec_scan)
    walk, _, pages, _ = _decode_one(dec, data)
    assert walk == 2 and pages == (n + 6) // 7
    data = W.write_file([W.Column("x", W.INT64, v, rows_per_page=300)], n)
    walk, _, pages, _ = _decode_one(dec_scan, data)
    assert walk == 0 and pages == (n + 299) // 300


def test_scan_garbage_lists_bounded(dec):
    # payload bytes that parse as a PageHeader prefix followed by a thrift list
    # header claiming ~2^31 elements: the candidate parse must stay bounded
    n = 200_000
    pat = np.frombuffer(bytes([0x15, 0x00, 0x15, 0x00, 0x19, 0xF5, 0xFF, 0xFF]), dtype=np.int64)[0]
    v = np.full(n, pat, dtype=np.int64)
    v[1::2] = 0x0101010101010101
    data = W.write_file([W.Column("x", W.INT64, v, rows_per_page=50_000)], n)
    P.compare_file(data, dec)


@pytest.mark.parametrize("w", [9, 11, 16, 17, 21, 24, 25, 31, 32])
def test_dict_index_widths(dec, w):
    # index streams wider than log2(dictionary size) are valid; mixed RLE / bit-packed runs
    rng = np.random.default_rng(w)
    d = 1000
    dvals = rng.integers(-2**31, 2**31 - 1, size=d).astype(np.int32)
    dpage = U.page_header_dict(4 * d, 4 * d, d) + dvals.tobytes()
    for min_rle in (3, 8, 1 << 30):
        keys = np.repeat(rng.integers(0, d, size=700), rng.integers(1, 12, size=700))[:3000].astype(np.uint32)
        idx = bytes([w]) + W.hybrid_encode(keys, w, min_rle=min_rle)
        P.compare_chunk_bytes(dpage + U.v1_page(idx, len(keys), 8), dec, ptype=abi.INT32)


# ---------------------------------------------------------------- K7: byte arrays
def test_c4_dict_then_plain_fallback(dec):
    # dictionary pages first, PLAIN pages after the dictionary fills (pyarrow-like),
    # SNAPPY, V1: chars and int64 offsets must match the oracle byte for byte
    import pqgpu
    data, _ = W.config_c4(rows=120_000, vocab=8192, rows_per_page=4000, dict_limit=100_000)
    res = P.compare_file(data, dec)
    assert res[0].status == 0 and res[0].value_width == 0
    pages = dec.pages(0)
    encs = [p.encoding for p in pages if p.page_type == 0]
    assert 8 in encs and 0 in encs, encs  # both page kinds present
    pf = pqgpu.ParquetFile(data)
    assert pf.columns[0].desc.physical_type == abi.BYTE_ARRAY


def test_c4_uncompressed_v2(dec):
    data, _ = W.config_c4(rows=50_000, vocab=3000, rows_per_page=7000, dict_limit=40_000, codec=W.UNCOMPRESSED)
    P.compare_file(data, dec)


def test_byte_array_plain_optional(dec):
    rng = np.random.default_rng(11)
    n = 30_000
    defs = (rng.random(n) >= 0.2).astype(np.uint8)
    nn = int(defs.sum())
    lens = rng.integers(0, 70, size=nn)
    lens[::13] = 0  # empty strings
    offs = np.zeros(nn + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    chars = rng.integers(0, 256, size=int(offs[-1]), dtype=np.uint8)
    for pv, codec in ((1, W.UNCOMPRESSED), (2, W.SNAPPY)):
        col = W.Column("s", W.BYTE_ARRAY, chars, offsets=offs, repetition=W.OPTIONAL, def_levels=defs,
                       rows_per_page=4000, page_version=pv, codec=codec)
        P.compare_file(W.write_file([col], n, row_groups=2), dec)


def test_byte_array_long_values(dec):
    # values longer than the 1 KiB walk window, and a page of a single value
    rng = np.random.default_rng(12)
    lens = np.array([5000, 1, 0, 1023, 1024, 1025, 3, 70000, 2], dtype=np.int64)
    offs = np.r_[0, np.cumsum(lens)].astype(np.int64)
    chars = rng.integers(0, 256, size=int(offs[-1]), dtype=np.uint8)
    for rpp in (1, 4, 9):
        col = W.Column("s", W.BYTE_ARRAY, chars, offsets=offs, rows_per_page=rpp)
        P.compare_file(W.write_file([col], len(lens)), dec)


def _str_cases():
    i32 = lambda a: np.array(a, dtype=np.int32).tobytes()  # noqa: E731
    u = U.u32
    H = W.hybrid_encode
    cases = []
    plain = u(3) + b"abc" + u(0) + u(5) + b"hello"
    cases.append(("ba_plain_ok", U.v1_page(plain, 3, 0), dict(ptype=abi.BYTE_ARRAY)))
    cases.append(("ba_plain_negative", U.v1_page(u(3) + b"abc" + i32([-1]) + b"zz", 2, 0), dict(ptype=abi.BYTE_ARRAY)))
    cases.append(("ba_plain_short_len", U.v1_page(u(3) + b"abc" + b"\x01\x00", 2, 0), dict(ptype=abi.BYTE_ARRAY)))
    cases.append(("ba_plain_short_chars", U.v1_page(u(3) + b"abc" + u(9) + b"abcd", 2, 0),
                  dict(ptype=abi.BYTE_ARRAY)))
    cases.append(("ba_plain_trailing", U.v1_page(plain + b"\x07\x07", 3, 0), dict(ptype=abi.BYTE_ARRAY)))
    cases.append(("ba_plain_all_empty", U.v1_page(u(0) * 100, 100, 0), dict(ptype=abi.BYTE_ARRAY)))
    cases.append(("flba0_plain", U.v1_page(plain, 3, 0), dict(ptype=abi.FIXED_LEN_BYTE_ARRAY, type_length=0)))
    # string dictionary
    dict_body = u(2) + b"xy" + u(0) + u(4) + b"wxyz"
    dpage = U.page_header_dict(len(dict_body), len(dict_body), 3) + dict_body
    idx = bytes([2]) + H([0, 1, 2, 2, 1, 0, 0, 2, 1, 1], 2)
    cases.append(("ba_dict_ok", dpage + U.v1_page(idx, 10, 8), dict(ptype=abi.BYTE_ARRAY)))
    cases.append(("ba_dict_then_plain", dpage + U.v1_page(idx, 10, 8) + U.v1_page(plain, 3, 0),
                  dict(ptype=abi.BYTE_ARRAY)))
    cases.append(("ba_dict_bad_index", dpage + U.v1_page(bytes([2]) + H([0, 3], 2), 2, 8),
                  dict(ptype=abi.BYTE_ARRAY)))
    cases.append(("ba_dict_zero_width", dpage + U.v1_page(bytes([0]), 4, 8), dict(ptype=abi.BYTE_ARRAY)))
    short = U.page_header_dict(len(dict_body), len(dict_body), 4) + dict_body  # 4 entries claimed, 3 present
    cases.append(("ba_dict_short", short + U.v1_page(bytes([2]) + H([3, 0], 2), 2, 8), dict(ptype=abi.BYTE_ARRAY)))
    negd = u(2) + b"xy" + i32([-5])
    cases.append(("ba_dict_negative", U.page_header_dict(len(negd), len(negd), 2) + negd
                  + U.v1_page(bytes([1]) + H([0], 1), 1, 8), dict(ptype=abi.BYTE_ARRAY)))
    cases.append(("ba_dict_nulls", dpage + U.v1_page(bytes([2]) + H([2, 0], 2), 4, 8, defs=H([1, 0, 0, 1], 1)),
                  dict(ptype=abi.BYTE_ARRAY, max_def=1)))
    # fixed-width short dictionary (advisor case): count > payload / width, index past the payload
    sd = U.page_header_dict(8, 8, 1000) + i32([1, 2])
    cases.append(("dict_short_fixed", sd + U.v1_page(bytes([10]) + H([999, 0], 10), 2, 8), dict(ptype=abi.INT32)))
    # zero bit width over a dictionary of 4097..79 872 entries (advisor case): the
    # page yields dict[0] for every value (hybrid_decoder.go:84-86), alone and
    # next to a page that does send its keys to the big-dictionary kernel
    bigd = np.arange(7, 7 + 5000, dtype=np.int32).tobytes()
    bdp = U.page_header_dict(len(bigd), len(bigd), 5000) + bigd
    cases.append(("dict_big_zero_width", bdp + U.v1_page(bytes([0]), 9, 8), dict(ptype=abi.INT32)))
    cases.append(("dict_big_zero_width_mixed", bdp + U.v1_page(bytes([0]), 9, 8)
                  + U.v1_page(bytes([13]) + H([4999, 0, 17, 4096], 13), 4, 8) + U.v1_page(bytes([0]), 3, 8),
                  dict(ptype=abi.INT32)))
    cases.append(("dict_big_zero_width_nulls", bdp + U.v1_page(bytes([0]), 6, 8, defs=H([1, 0, 1, 1, 0, 1], 1)),
                  dict(ptype=abi.INT32, max_def=1)))
    return cases


@pytest.mark.parametrize("case", _str_cases(), ids=lambda c: c[0])
def test_byte_array_hand_built(dec, case):
    name, chunk, kw = case
    P.compare_chunk_bytes(chunk, dec, **kw)


def test_capacity_grows_once_then_remembered(dec):
    """A chunk the planner under-sizes (no num_values hint, tiny pages, string
    dictionary) grows its arenas over several attempts in the first call; the
    second call reuses the learned capacities and launches the pipeline once."""
    import pqgpu
    rng = np.random.default_rng(13)
    n = 30_000
    lens = rng.integers(0, 40, size=n)
    offs = np.r_[0, np.cumsum(lens)].astype(np.int64)
    vocab = rng.integers(97, 123, size=int(offs[-1]), dtype=np.uint8)
    col = W.Column("s", W.BYTE_ARRAY, vocab, offsets=offs, encoding=W.RLE_DICTIONARY, rows_per_page=50)
    data = W.write_file([col], n)
    pf = pqgpu.ParquetFile(data)
    dev = dec.upload(pf.data)
    try:
        job = pqgpu.device_job(pf, 0, 0, dev)
        job.num_values_hint = 0
        job.total_uncompressed_size = 0
        exp = P.oracle_chunk(pf, 0, 0)
        r = dec.decode_jobs([job])[0]
        first = dec.debug_job(0)[4]
        P.compare_chunk(exp, dec.download(r, 0), "first call")
        r = dec.decode_jobs([job])[0]
        second = dec.debug_job(0)[4]
        P.compare_chunk(exp, dec.download(r, 0), "second call")
        assert first >= 3 and second == 1, (first, second)
    finally:
        dec.free(dev)


# ---------------------------------------------------------------- C5: nested list + 8 mixed columns
def test_c5_every_column(dec):
    """Reduced-row C5 (LIST<double> + 8 mixed columns, 3 row groups): every
    chunk of every row group against the oracle."""
    data, _ = W.config_c5(row_groups=(0, 31, 63), rows_per_rg=45_000)
    res = P.compare_file(data, dec)
    assert len(res) == 27 and all(r.status == 0 for r in res)


def test_c5_single_page_chunks(dec):
    """parquet-go's own writer puts one data page in each chunk (chunk_writer.go:237-246)."""
    data, _ = W.config_c5(row_groups=(5,), rows_per_rg=30_000, rows_per_page=30_000)
    P.compare_file(data, dec)


def test_byte_array_chain_guesses_wrong(dec):
    """PLAIN byte arrays whose bytes look like length prefixes everywhere (zero
    bytes, embedded u32 lengths): the segment walks start at wrong guesses and
    the in-order check must re-walk them; big pages span hundreds of segments."""
    rng = np.random.default_rng(21)
    n = 60_000
    for kind in ("zeros", "fake_prefix", "mixed"):
        lens = rng.integers(0, 24, size=n)
        offs = np.r_[0, np.cumsum(lens)].astype(np.int64)
        if kind == "zeros":
            chars = np.zeros(int(offs[-1]), np.uint8)
        elif kind == "fake_prefix":
            pat = np.frombuffer(np.array([4, 8, 0, 3], dtype=np.uint32).tobytes(), np.uint8)
            chars = np.resize(pat, int(offs[-1]))
        else:
            chars = rng.integers(0, 3, size=int(offs[-1])).astype(np.uint8)
        for rpp in (n, 7000):
            col = W.Column("s", W.BYTE_ARRAY, chars, offsets=offs, rows_per_page=rpp)
            P.compare_file(W.write_file([col], n), dec)
    # a string dictionary of such entries, then a corrupt tail inside a big page
    col = W.Column("s", W.BYTE_ARRAY, np.zeros(int(offs[-1]), np.uint8), offsets=offs, rows_per_page=n)
    data = bytearray(W.write_file([col], n))
    import pqgpu
    pf = pqgpu.ParquetFile(bytes(data))
    m = pf.chunk_meta(0, 0)
    for at, val in ((m.start + m.total_compressed_size - 9, 0xFF), (m.start + m.total_compressed_size // 2, 0x80)):
        b = bytearray(data)
        b[at] = val
        P.compare_file(bytes(b), dec)


def test_delta_block_lengths_vary(dec):
    """The speculative DBP header walk (pqg_values.hip dbp_decode): stretches of
    equal-length blocks broken by blocks of other widths and other min-delta
    varint lengths, and a ragged last block."""
    rng = np.random.default_rng(11)
    parts = []
    for k, (nb, lo, hi) in enumerate([(40, 950, 1051), (3, 0, 1 << 20), (1, -5, 6), (70, 950, 1051), (2, 10**6, 10**6 + 3),
                                      (1, -(1 << 40), 1 << 40), (30, 950, 1051)]):
        parts.append(rng.integers(lo, hi, size=nb * 128 + (k == 6) * 57, dtype=np.int64))
    v = np.cumsum(np.concatenate(parts))
    for codec, ver in ((W.UNCOMPRESSED, 1), (W.SNAPPY, 2)):
        data = W.write_file([W.Column("d", W.INT64, v, encoding=W.DELTA_BINARY_PACKED, rows_per_page=len(v),
                                      codec=codec, page_version=ver)], len(v))
        P.compare_file(data, dec)
        v32 = (v & 0x7FFFFFFF).astype(np.int32)
        data = W.write_file([W.Column("d", W.INT32, v32, encoding=W.DELTA_BINARY_PACKED, rows_per_page=len(v32),
                                      codec=codec, page_version=ver)], len(v32))
        P.compare_file(data, dec)


def test_delta_corrupt_bytes_match(dec):
    """One byte of a DBP page's block headers overwritten — a width past the
    type's bits (0x41, 0xFF), a width that changes the block's length (8, 0),
    a min delta one varint byte longer — at blocks inside and at the edges of
    the speculative walk's 64-header groups: GPU and oracle agree on the
    status and on every value."""
    rng = np.random.default_rng(12)
    v = np.cumsum(1000 + rng.integers(-50, 51, size=150 * 128, dtype=np.int64))
    base = W.write_file([W.Column("d", W.INT64, v, encoding=W.DELTA_BINARY_PACKED, rows_per_page=len(v))], len(v))
    # every block here is [2-byte min delta][widths 7 7 7 7][4 x 28 bytes]
    at = [i for i in range(len(base) - 3) if base[i:i + 4] == b"\x07\x07\x07\x07"]
    heads = [a for a, b in zip(at, at[1:]) if b - a == 118] + [at[-1]]
    assert len(heads) >= 140
    statuses = set()
    for blk in (1, 2, 37, 63, 64, 65, 100, 127, 128, len(heads) - 1):
        w = heads[blk]
        for pos, byte in ((w + 1, 0x41), (w + 3, 0xFF), (w, 8), (w + 2, 0), (w - 2, base[w - 2] | 0x80)):
            data = bytearray(base)
            data[pos] = byte
            statuses.add(P.compare_file(bytes(data), dec)[0].status)
    assert len(statuses) > 1  # errors were reached, not only silent value changes
