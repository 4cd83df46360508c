"""Big pages: parquet-go's own writer puts a whole column chunk into ONE data
page (chunk_writer.go:237-246) and writes every level / dictionary-index
stream as one bit-packed run (hybridEncoder.bpEncode, hybrid_encoder.go:59-73).
libpqgpu cuts such pages into parts decoded by many waves (k_part_plan), and
hands long runs of the serial walks to parallel kernels (k_level_long,
k_walk_long).  GPU vs oracle, bit-exact, on single pages of >= 1M values of
each encoding the split touches, plus the edges: a bad dictionary key in a
middle part, a zero-padded short last group (Q5) inside a long level run,
pyarrow-style runs in a big page, and a part boundary inside a multi-run
block."""
import numpy as np
import pytest

import parity as P
import pqtest_util as U
from gen import pqwrite as W
from pqgpu import abi

pytestmark = pytest.mark.gpu
REF = dict(hybrid_groups=W.REF_HYBRID)


@pytest.fixture(scope="module")
def dec():
    import pqgpu
    d = pqgpu.GpuDecoder(0)
    yield d
    d.close()


def one_page(cols, rows):
    for c in cols:
        c.rows_per_page = rows
    return W.write_file(cols, rows)


def test_plain_int64_one_page(dec):
    rows = 1_000_003
    v = W.splitmix64(1, rows).view(np.int64)
    P.compare_file(one_page([W.Column("a", W.INT64, v)], rows), dec)


def test_plain_fixed_types_one_page(dec):
    rng = np.random.default_rng(2)
    rows = 1_100_000
    cols = [W.Column("f", W.FLOAT, rng.standard_normal(rows).astype(np.float32)),
            W.Column("b", W.BOOLEAN, rng.integers(0, 2, rows).astype(np.uint8)),
            W.Column("i96", W.INT96, rng.integers(0, 256, size=rows * 12, dtype=np.uint8)),
            W.Column("fx", W.FLBA, rng.integers(0, 256, size=rows * 3, dtype=np.uint8), type_length=3)]
    P.compare_file(one_page(cols, rows), dec)


@pytest.mark.parametrize("null_frac", [0.1, 0.0])
def test_optional_plain_ref_levels(dec, null_frac):
    rng = np.random.default_rng(3)
    rows = 1_200_000
    defs = (rng.random(rows) >= null_frac).astype(np.uint8)
    v = rng.integers(-2**31, 2**31 - 1, size=int(defs.sum()), dtype=np.int64).astype(np.int32)
    col = W.Column("o", W.INT32, v, repetition=W.OPTIONAL, def_levels=defs, **REF)
    res = P.compare_file(one_page([col], rows), dec)
    assert res[0].num_values == int(defs.sum())


def test_list_double_ref_levels(dec):
    parts = W.c5_row_group_columns(0, 600_000)
    e = parts["lst"]
    col = W.Column("lst", W.DOUBLE, e["values"], repetition=W.LIST, def_levels=e["def_levels"],
                   rep_levels=e["rep_levels"], **REF)
    P.compare_file(one_page([col], 600_000), dec)


@pytest.mark.parametrize("bits,null_frac", [(12, 0.1), (20, 0.0), (3, 0.3)])
def test_dict_int32_ref_one_page(dec, bits, null_frac):
    rows = 1_000_000
    data, _ = W.config_c2(rows=rows, bits=bits, null_frac=null_frac, rows_per_page=rows)
    P.compare_file(data, dec)  # pyarrow-like runs (<= 64 groups): parts at block starts
    rng = np.random.default_rng(bits)
    d = 1 << bits
    defs = (rng.random(rows) >= null_frac).astype(np.uint8)
    dv = rng.integers(-2**31, 2**31 - 1, size=d, dtype=np.int64).astype(np.int32)
    idx = rng.integers(0, d, size=int(defs.sum()))
    idx[:d] = np.arange(min(d, len(idx)))
    col = W.Column("c", W.INT32, dv[idx], repetition=W.OPTIONAL, def_levels=defs, encoding=W.RLE_DICTIONARY, **REF)
    P.compare_file(one_page([col], rows), dec)


def test_dict_run_heavy_one_page(dec):
    rows = 1_000_000
    data, _ = W.config_c2(rows=rows, bits=8, run_heavy=True, rows_per_page=rows)
    P.compare_file(data, dec)


def test_dict_int64_and_double_one_page(dec):
    rng = np.random.default_rng(9)
    rows = 1_050_000
    cols = [W.Column("di", W.INT64, rng.integers(0, 3000, rows), encoding=W.RLE_DICTIONARY, **REF),
            W.Column("dd", W.DOUBLE, rng.integers(0, 50, rows).astype(np.float64), encoding=W.RLE_DICTIONARY)]
    P.compare_file(one_page(cols, rows), dec)


def _strings(rows, vocab, seed):
    rng = np.random.default_rng(seed)
    chars, offs = W.make_vocab(vocab, seed)
    keys = rng.integers(0, vocab, size=rows)
    lens = (offs[1:] - offs[:-1])[keys]
    so = np.zeros(rows + 1, np.int64)
    so[1:] = np.cumsum(lens)
    idx = np.repeat(offs[:-1][keys] - so[:-1], lens) + np.arange(int(so[-1]), dtype=np.int64)
    return chars[idx], so


def test_string_dict_ref_one_page(dec):
    rows = 1_000_000
    ch, so = _strings(rows, 4096, 5)
    col = W.Column("s", W.BYTE_ARRAY, ch, offsets=so, encoding=W.RLE_DICTIONARY, **REF)
    P.compare_file(one_page([col], rows), dec)


def test_string_plain_one_page(dec):
    rows = 300_000
    ch, so = _strings(rows, 5000, 6)
    col = W.Column("s", W.BYTE_ARRAY, ch, offsets=so, encoding=W.PLAIN)
    P.compare_file(one_page([col], rows), dec)


def test_c5_one_page_columns(dec):
    """The C5 layout at 300 000 rows per row group: lst, oi32 and s are one
    page per chunk (parquet-go's writer), two row groups."""
    data, _ = W.config_c5(row_groups=(0, 1), rows_per_rg=300_000)
    P.compare_file(data, dec)


def test_delta_one_page(dec):
    rows = 1_000_001  # (N - 1) % 128 == 0 would be Q3: N - 1 = 1 000 000 = 7812 * 128 + 64
    v = np.cumsum(np.random.default_rng(4).integers(-1000, 1000, rows))
    data = one_page([W.Column("d", W.INT64, v, encoding=W.DELTA_BINARY_PACKED)], rows)
    P.compare_file(data, dec)


def _single_run_dict_chunk(n, d, w, bad_at=None):
    """A dictionary chunk of one V1 page: d int32 entries, n required keys as
    one bit-packed run (the reference writer's layout); key `bad_at` set to
    2^w - 1 (>= d: "dict: invalid index")."""
    rng = np.random.default_rng(12)
    dvals = rng.integers(-2**31, 2**31 - 1, size=d, dtype=np.int64).astype(np.int32)
    keys = rng.integers(0, d, size=n).astype(np.uint32)
    if bad_at is not None:
        keys[bad_at] = (1 << w) - 1
    stream = bytes([w]) + U.uvarint(((n + 7) // 8) << 1 | 1)
    bits = np.zeros(((n + 7) // 8) * 8 * w, np.uint8)
    for k in range(w):
        bits[k::w][:n] = (keys >> k) & 1
    stream += np.packbits(bits, bitorder="little").tobytes()
    dict_body = dvals.tobytes()
    dp = U.page_header_dict(len(dict_body), len(dict_body), d) + dict_body
    page = U.v1_page(stream, n, abi.ENC_RLE_DICTIONARY)
    return dp + page, len(dp)


@pytest.mark.parametrize("bad_at", [None, 0, 700_001, 1_199_999])
def test_dict_bad_key_in_a_part(dec, bad_at):
    chunk, dpo = _single_run_dict_chunk(1_200_000, 3000, 12, bad_at)
    exp, got = P.compare_chunk_bytes(chunk, dec, ptype=abi.INT32, data_page_offset=dpo, has_dict_off=True)
    assert exp.status == (0 if bad_at is None else abi.STATUS_CODES["DICT_INDEX"])


def test_long_level_run_short_last_group(dec):
    """maxD 3 (w = 2) def levels of 200 000 values as one bit-packed run whose
    length prefix drops the last byte: the last group starts inside the stream
    and reads zero past its end (Q5, hybrid_decoder.go:133-141)."""
    n = 200_000
    rng = np.random.default_rng(7)
    lv = rng.integers(0, 4, size=n).astype(np.uint32)
    lv[-3:] = 3
    groups = (n + 7) // 8
    bits = np.zeros(groups * 8 * 2, np.uint8)
    bits[0::2][:n] = lv & 1
    bits[1::2][:n] = (lv >> 1) & 1
    run = U.uvarint(groups << 1 | 1) + np.packbits(bits, bitorder="little").tobytes()
    run = run[:-1]  # the short last group
    vals = np.zeros(n, np.float64)
    body = U.u32(len(run)) + run + vals.tobytes()
    chunk = U.page_header_v1(len(body), len(body), n, abi.ENC_PLAIN) + body
    exp, got = P.compare_chunk_bytes(chunk, dec, ptype=abi.DOUBLE, max_def=3)
    assert exp.status == 0
