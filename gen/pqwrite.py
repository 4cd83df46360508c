"""Python front-end of the synthetic parquet writer (gen/libpqwrite.so).

Test/bench input generation only.  `Column` describes one leaf column with its
dense non-null values and (optional) def/rep levels; `write_file` returns the
file bytes.  `config_*` build the BASELINE configs C1..C5 at any scale.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

BOOLEAN, INT32, INT64, INT96, FLOAT, DOUBLE, BYTE_ARRAY, FLBA = range(8)
PLAIN, RLE_DICTIONARY, DELTA_BINARY_PACKED = 0, 8, 5
DELTA_LENGTH_BYTE_ARRAY, DELTA_BYTE_ARRAY = 6, 7
UNCOMPRESSED, SNAPPY, GZIP = 0, 1, 2
REQUIRED, OPTIONAL, LIST = 0, 1, 2
REF_HYBRID = -1  # Column(hybrid_groups=...): parquet-go's writer layout (one bit-packed run per stream)

_lib = None


class _PqwColumn(C.Structure):
    _fields_ = [
        ("name", C.c_char_p),
        ("type", C.c_int32), ("type_length", C.c_int32), ("repetition", C.c_int32),
        ("encoding", C.c_int32), ("codec", C.c_int32), ("page_version", C.c_int32),
        ("rows_per_page", C.c_int32), ("min_rle", C.c_int32),
        ("v2_uncompressed_flag", C.c_int32), ("hybrid_groups", C.c_int32),
        ("dict_limit", C.c_int64),
        ("values", C.c_void_p), ("offsets", C.c_void_p),
        ("def_levels", C.c_void_p), ("rep_levels", C.c_void_p),
        ("num_slots", C.c_int64), ("num_values", C.c_int64),
    ]


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "libpqwrite.so")
        if not os.path.exists(path):
            raise RuntimeError("writer not built: run `make -C gen`")
        L = C.CDLL(path)
        L.pqw_write_file.argtypes = [C.POINTER(_PqwColumn), C.c_int, C.c_int64, C.c_int,
                                     C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]
        L.pqw_free.argtypes = [C.c_void_p]
        L.pqw_hybrid_encode.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_void_p, C.c_int64]
        L.pqw_hybrid_encode.restype = C.c_int64
        L.pqw_dbp_encode64.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64]
        L.pqw_dbp_encode64.restype = C.c_int64
        L.pqw_dbp_encode32.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64]
        L.pqw_dbp_encode32.restype = C.c_int64
        L.pqw_snappy_compress.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64]
        L.pqw_snappy_compress.restype = C.c_int64
        L.pqw_set_snappy_block.argtypes = [C.c_int64]
        L.pqw_set_snappy_block.restype = None
        L.pqw_writer_new.argtypes = []
        L.pqw_writer_new.restype = C.c_void_p
        L.pqw_writer_add.argtypes = [C.c_void_p, C.POINTER(_PqwColumn), C.c_int, C.c_int64]
        L.pqw_writer_finish.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]
        L.pqw_writer_free.argtypes = [C.c_void_p]
        L.pqw_writer_free.restype = None
        _lib = L
    return _lib


class Column:
    def __init__(self, name, ptype, values, *, type_length=0, repetition=REQUIRED, encoding=PLAIN,
                 codec=UNCOMPRESSED, page_version=1, rows_per_page=20000, def_levels=None,
                 rep_levels=None, offsets=None, dict_limit=0, min_rle=8, v2_uncompressed_flag=False,
                 hybrid_groups=0):
        self.name = name
        self.ptype = ptype
        self.type_length = type_length
        self.repetition = repetition
        self.encoding = encoding
        self.codec = codec
        self.page_version = page_version
        self.rows_per_page = rows_per_page
        self.min_rle = min_rle
        self.dict_limit = dict_limit
        self.v2_uncompressed_flag = v2_uncompressed_flag
        # literal groups per bit-packed run of the level / index streams: 0 = 64
        # (pyarrow-like); REF_HYBRID = one bit-packed run per stream, as
        # parquet-go's hybridEncoder writes them (hybrid_encoder.go:59-99)
        self.hybrid_groups = hybrid_groups
        self.values = np.ascontiguousarray(values)
        self.offsets = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.int64)
        self.def_levels = None if def_levels is None else np.ascontiguousarray(def_levels, dtype=np.uint8)
        self.rep_levels = None if rep_levels is None else np.ascontiguousarray(rep_levels, dtype=np.uint8)
        if self.offsets is not None:
            self.num_values = len(self.offsets) - 1
        elif ptype == FLBA:
            self.num_values = self.values.nbytes // type_length
        elif ptype == INT96:
            self.num_values = self.values.nbytes // 12
        else:
            self.num_values = len(self.values)
        self.num_slots = len(self.def_levels) if self.def_levels is not None else self.num_values

    @property
    def max_def(self):
        return {REQUIRED: 0, OPTIONAL: 1, LIST: 3}[self.repetition]

    @property
    def max_rep(self):
        return 1 if self.repetition == LIST else 0


def _pqw_columns(columns):
    arr = (_PqwColumn * len(columns))()
    names = []
    for i, c in enumerate(columns):
        names.append(c.name.encode())
        a = arr[i]
        a.name = names[-1]
        a.type, a.type_length, a.repetition = c.ptype, c.type_length, c.repetition
        a.encoding, a.codec, a.page_version = c.encoding, c.codec, c.page_version
        a.rows_per_page, a.min_rle = c.rows_per_page, c.min_rle
        a.v2_uncompressed_flag = int(c.v2_uncompressed_flag)
        a.hybrid_groups = c.hybrid_groups
        a.dict_limit = c.dict_limit
        a.values = c.values.ctypes.data if c.values.size else None
        a.offsets = c.offsets.ctypes.data if c.offsets is not None else None
        a.def_levels = c.def_levels.ctypes.data if c.def_levels is not None else None
        a.rep_levels = c.rep_levels.ctypes.data if c.rep_levels is not None else None
        a.num_slots, a.num_values = c.num_slots, c.num_values
    return arr, names


def write_file(columns, num_rows, row_groups=1):
    L = lib()
    arr, names = _pqw_columns(columns)
    out = C.c_void_p()
    n = C.c_int64()
    rc = L.pqw_write_file(arr, len(columns), num_rows, row_groups, C.byref(out), C.byref(n))
    if rc != 0:
        raise ValueError("pqw_write_file failed: %d" % rc)
    # (ctypes.string_at takes a C int size: files past 2 GiB are copied via numpy)
    data = np.ctypeslib.as_array(C.cast(out, C.POINTER(C.c_uint8)), shape=(n.value,)).tobytes()
    L.pqw_free(out)
    return data


class RowGroupWriter:
    """A file written one row group at a time (pqw_writer_*): the caller builds
    one row group's columns, add()s them and drops them, so it never holds
    more than one row group's arrays.  finish() returns the file as a numpy
    uint8 array (one copy of the bytes; ParquetFile takes it without copying)."""

    def __init__(self):
        self._h = lib().pqw_writer_new()

    def add(self, columns, num_rows):
        arr, names = _pqw_columns(columns)
        rc = lib().pqw_writer_add(self._h, arr, len(columns), num_rows)
        if rc != 0:
            raise ValueError("pqw_writer_add failed: %d" % rc)

    def finish(self):
        import weakref
        L = lib()
        out = C.c_void_p()
        n = C.c_int64()
        rc = L.pqw_writer_finish(self._h, C.byref(out), C.byref(n))
        self._h = None
        if rc != 0:
            raise ValueError("pqw_writer_finish failed: %d" % rc)
        # the writer's own buffer, freed when the array (and every view of it) is gone
        arr = np.ctypeslib.as_array(C.cast(out, C.POINTER(C.c_uint8)), shape=(n.value,))
        weakref.finalize(arr, L.pqw_free, out.value)
        return arr

    def __del__(self):
        if getattr(self, "_h", None):
            lib().pqw_writer_free(self._h)
            self._h = None


def hybrid_encode(values, width, min_rle=8):
    v = np.ascontiguousarray(values, dtype=np.uint32)
    cap = len(v) * 8 + 64
    out = np.zeros(cap, dtype=np.uint8)
    n = lib().pqw_hybrid_encode(v.ctypes.data, len(v), width, min_rle, out.ctypes.data, cap)
    assert n >= 0
    return out[:n].tobytes()


def dbp_encode(values, bits=64):
    v = np.ascontiguousarray(values, dtype=np.int64 if bits == 64 else np.int32)
    cap = len(v) * 10 + 1024
    out = np.zeros(cap, dtype=np.uint8)
    fn = lib().pqw_dbp_encode64 if bits == 64 else lib().pqw_dbp_encode32
    n = fn(v.ctypes.data, len(v), out.ctypes.data, cap)
    assert n >= 0
    return out[:n].tobytes()


SNAPPY_BLOCK = 65536  # golang/snappy maxBlockSize (snappy.go:72)


class snappy_block_size:
    """Inside `with snappy_block_size(0):` the writer compresses every snappy page
    as one block (copies across 64 KiB boundaries) instead of golang/snappy's
    independent 64 KiB blocks (the default, encode.go:18-41)."""

    def __init__(self, bs):
        self.bs = bs

    def __enter__(self):
        lib().pqw_set_snappy_block(self.bs)
        return self

    def __exit__(self, *a):
        lib().pqw_set_snappy_block(65536)


def snappy_compress(data: bytes):
    src = np.frombuffer(data, dtype=np.uint8)
    cap = len(data) + len(data) // 6 + 64
    out = np.zeros(cap, dtype=np.uint8)
    n = lib().pqw_snappy_compress(src.ctypes.data if len(src) else None, len(src), out.ctypes.data, cap)
    assert n >= 0
    return out[:n].tobytes()


# --------------------------------------------------------------------------
# BASELINE configs (BASELINE.md "Configs as concrete synthetic inputs")
# --------------------------------------------------------------------------

def splitmix64(seed, n):
    x = (np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(seed))
    z = x.copy()
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def config_c1(rows=10_000_000, rows_per_page=20000, seed=1):
    """C1: required int64, PLAIN, UNCOMPRESSED, one row group, V1."""
    vals = splitmix64(seed, rows).view(np.int64)
    col = Column("c1", INT64, vals, rows_per_page=rows_per_page)
    return write_file([col], rows), {"rows": rows, "values": vals}


def config_c2(rows=100_000_000, bits=8, null_frac=0.10, run_heavy=False, rows_per_page=20000, seed=2,
              page_version=1, codec=UNCOMPRESSED):
    """C2: optional int32, RLE_DICTIONARY with D = 2^bits entries, ~10% nulls, V1."""
    rng = np.random.default_rng(seed + bits)
    d = 1 << bits
    dict_vals = rng.integers(-2**31, 2**31 - 1, size=d, dtype=np.int64).astype(np.int32)
    dict_vals[: min(d, 1)] = 0
    defs = (rng.random(rows) >= null_frac).astype(np.uint8)
    nn = int(defs.sum())
    if run_heavy:
        lens = rng.geometric(1.0 / 16, size=nn // 4 + 16)
        keys = rng.integers(0, d, size=len(lens))
        idx = np.repeat(keys, lens)[:nn]
        if len(idx) < nn:
            idx = np.concatenate([idx, rng.integers(0, d, size=nn - len(idx))])
    else:
        idx = rng.integers(0, d, size=nn)
        # make sure every dictionary entry appears so the index width is `bits`
        idx[: min(d, nn)] = np.arange(min(d, nn))
    vals = dict_vals[idx]
    col = Column("c2", INT32, vals, repetition=OPTIONAL, encoding=RLE_DICTIONARY, def_levels=defs,
                 rows_per_page=rows_per_page, page_version=page_version, codec=codec)
    return write_file([col], rows), {"rows": rows, "non_null": nn, "bits": bits}


def config_c3(rows=200_000_000, rows_per_page=20000, seed=3, codec=SNAPPY):
    """C3: int64 timestamps, DELTA_BINARY_PACKED, V2, SNAPPY (is_compressed=true)."""
    rng = np.random.default_rng(seed)
    deltas = 1000 + rng.integers(-50, 51, size=rows, dtype=np.int64)
    deltas[0] = 0
    vals = np.int64(1_600_000_000_000_000) + np.cumsum(deltas)
    col = Column("ts", INT64, vals, encoding=DELTA_BINARY_PACKED, codec=codec, page_version=2,
                 rows_per_page=rows_per_page)
    return write_file([col], rows), {"rows": rows, "values": vals}


def make_vocab(n, seed, lo=4, hi=32):
    rng = np.random.default_rng(seed)
    lens = rng.integers(lo, hi + 1, size=n)
    offs = np.zeros(n + 1, dtype=np.int64)
    offs[1:] = np.cumsum(lens)
    chars = rng.integers(97, 123, size=int(offs[-1]), dtype=np.uint8)
    # make words unique by stamping the index into the first 4 bytes
    for i in range(n):
        chars[offs[i]:offs[i] + 4] = np.frombuffer(np.uint32(i).tobytes(), dtype=np.uint8) % 26 + 65
    return chars, offs


def config_c4(rows=50_000_000, vocab=65536, rows_per_page=20000, seed=4, dict_limit=1 << 20, codec=SNAPPY):
    """C4: required STRING, dictionary then PLAIN fallback after 1 MiB of dictionary, SNAPPY, V1."""
    rng = np.random.default_rng(seed)
    chars, offs = make_vocab(vocab, seed)
    ranks = rng.zipf(1.1, size=rows * 2)
    ranks = ranks[ranks <= vocab][:rows] - 1
    while len(ranks) < rows:
        more = rng.zipf(1.1, size=rows)
        ranks = np.concatenate([ranks, more[more <= vocab][: rows - len(ranks)] - 1])
    lens = (offs[1:] - offs[:-1])[ranks]
    out_offs = np.zeros(rows + 1, dtype=np.int64)
    out_offs[1:] = np.cumsum(lens)
    starts = offs[:-1][ranks]
    total = int(out_offs[-1])
    # gather chars, 2 M rows at a time (a whole-column index array would be
    # 8 bytes per char, ~20 GB of host memory at 50 M rows)
    out_chars = np.empty(total, dtype=np.uint8)
    step = 1 << 21
    for r0 in range(0, rows, step):
        r1 = min(rows, r0 + step)
        c0, c1 = int(out_offs[r0]), int(out_offs[r1])
        idx = np.repeat(starts[r0:r1] - out_offs[r0:r1], lens[r0:r1]) + np.arange(c0, c1, dtype=np.int64)
        out_chars[c0:c1] = chars[idx]
    del idx
    col = Column("s", BYTE_ARRAY, out_chars, offsets=out_offs, encoding=RLE_DICTIONARY, codec=codec,
                 rows_per_page=rows_per_page, dict_limit=dict_limit)
    return write_file([col], rows), {"rows": rows, "chars": out_chars, "offsets": out_offs}


def config_delta_strings(rows=200_000, encoding=DELTA_BYTE_ARRAY, rows_per_page=20000, seed=6, codec=SNAPPY,
                         page_version=1, null_frac=0.0, sorted_values=True):
    """STRING column written with DELTA_LENGTH_BYTE_ARRAY or DELTA_BYTE_ARRAY
    (type_bytearray.go:98-240): values drawn from a vocabulary, sorted so that
    neighbours share prefixes (the shape DELTA_BYTE_ARRAY is for), optional
    nulls.  -> (file bytes, {"chars", "offsets", "defs"})."""
    rng = np.random.default_rng(seed)
    chars, offs = make_vocab(4096, seed)
    words = [bytes(chars[offs[i]:offs[i + 1]]) for i in range(len(offs) - 1)]
    prefixes = [b"http://example.com/", b"user_", b"", b"2024-01-"]
    nn_rows = rows
    defs = None
    if null_frac > 0:
        defs = (rng.random(rows) >= null_frac).astype(np.uint8)
        nn_rows = int(defs.sum())
    vals = [prefixes[int(rng.integers(0, len(prefixes)))] + words[int(rng.integers(0, len(words)))]
            for _ in range(nn_rows)]
    if sorted_values:
        vals.sort()
    out_offs = np.zeros(nn_rows + 1, dtype=np.int64)
    out_offs[1:] = np.cumsum([len(v) for v in vals])
    out_chars = np.frombuffer(b"".join(vals), dtype=np.uint8).copy() if vals else np.zeros(0, np.uint8)
    col = Column("s", BYTE_ARRAY, out_chars, offsets=out_offs, encoding=encoding, codec=codec,
                 rows_per_page=rows_per_page, page_version=page_version,
                 repetition=OPTIONAL if defs is not None else REQUIRED, def_levels=defs)
    return write_file([col], rows), {"chars": out_chars, "offsets": out_offs, "defs": defs}


def config_c2_family(rows=100_000_000, bits_list=(1, 2, 4, 8, 12, 16, 20), null_frac=0.10, rows_per_page=20000,
                     seed=2, run_heavy=False):
    """C2 at every index width: one file per width sharing the null pattern and
    the (masked) index draw.  Index streams: uniform keys
    (bit-packed dominated), or run_heavy: keys repeated in runs of geometric
    length, mean 16 (RLE runs dominate).  Yields (bits, file_bytes, expected)
    where expected = (def_levels u8[rows], dense int32 values)."""
    rng = np.random.default_rng(seed)
    defs = (rng.random(rows) >= null_frac).astype(np.uint8)
    nn = int(defs.sum())
    if run_heavy:
        lens = rng.geometric(1.0 / 16, size=nn // 8 + 64)
        while int(lens.sum()) < nn:
            lens = np.concatenate([lens, rng.geometric(1.0 / 16, size=nn // 16 + 64)])
        keys = rng.integers(0, 1 << 20, size=len(lens), dtype=np.int64)
        raw = np.repeat(keys, lens)[:nn]
    else:
        raw = rng.integers(0, 1 << 20, size=nn, dtype=np.int64)
    dict_all = rng.integers(-2**31, 2**31 - 1, size=1 << 20, dtype=np.int64).astype(np.int32)
    for bits in bits_list:
        d = 1 << bits
        idx = raw & (d - 1)
        idx[: min(d, nn)] = np.arange(min(d, nn))
        vals = dict_all[:d][idx]
        col = Column("c2", INT32, vals, repetition=OPTIONAL, encoding=RLE_DICTIONARY, def_levels=defs,
                     rows_per_page=rows_per_page)
        yield bits, write_file([col], rows), (defs, vals)


C5_ROWS_PER_RG = 15_625_000


def _dbp_safe_rows_per_page(rows, rows_per_page):
    """A page size whose pages all avoid the reference's DBP quirk Q3
    (N == 1 or (N - 1) % 128 == 0 fails with EOF, deltabp_decoder.go:114-175)."""
    bad = lambda n: n == 1 or (n - 1) % 128 == 0  # noqa: E731
    rpp = rows_per_page
    while bad(rpp) or (rows % rpp and bad(rows % rpp)):
        rpp += 1
    return rpp


def c5_row_group_columns(rg, rows, seed=5, rows_per_page=20000):
    """Column arrays of C5 row group `rg` (seeded by its global index, so any
    subset of the 64 row groups can be generated independently):
      lst   LIST<double> (3-level; length U{0..3}, 5% null lists, 5% null elements)
      i32   int32 PLAIN          i64d  int64 DELTA_BINARY_PACKED
      f64   double PLAIN         f32   float PLAIN
      i96   int96 PLAIN          oi32  optional int32 PLAIN (10% nulls, dictionary off: SURVEY §8d)
      s     required string RLE_DICTIONARY (4096-word vocabulary, length U[4,32])
      i64s  int64 PLAIN SNAPPY
    Returns a dict name -> dict(values, def_levels, rep_levels, offsets)."""
    rng = np.random.default_rng([seed, rg])
    out = {}
    # ---- LIST<double>
    null_list = rng.random(rows) < 0.05
    lens = rng.integers(0, 4, size=rows)
    lens[null_list] = 0
    per_row = np.where(lens == 0, 1, lens)
    starts = np.zeros(rows + 1, np.int64)
    starts[1:] = np.cumsum(per_row)
    slots = int(starts[-1])
    rep = np.ones(slots, np.uint8)
    rep[starts[:-1]] = 0
    row_of = np.repeat(np.arange(rows), per_row)
    defs = np.full(slots, 3, np.uint8)
    defs[rng.random(slots) < 0.05] = 2
    empty = (lens == 0)[row_of]
    defs[empty] = 1
    defs[null_list[row_of]] = 0
    nv = int((defs == 3).sum())
    out["lst"] = dict(values=rng.standard_normal(nv), def_levels=defs, rep_levels=rep)
    out["i32"] = dict(values=rng.integers(-2**31, 2**31 - 1, size=rows, dtype=np.int64).astype(np.int32))
    steps = rng.integers(-1000, 1000, size=rows, dtype=np.int64)
    out["i64d"] = dict(values=np.int64(rg) * 10**12 + np.cumsum(steps))
    out["f64"] = dict(values=rng.standard_normal(rows))
    out["f32"] = dict(values=rng.standard_normal(rows).astype(np.float32))
    out["i96"] = dict(values=rng.integers(0, 256, size=rows * 12, dtype=np.uint8))
    od = (rng.random(rows) >= 0.10).astype(np.uint8)
    dvals = rng.integers(-2**31, 2**31 - 1, size=1000, dtype=np.int64).astype(np.int32)
    out["oi32"] = dict(values=dvals[rng.integers(0, 1000, size=int(od.sum()))], def_levels=od)
    chars, offs = make_vocab(4096, seed)
    keys = rng.integers(0, 4096, size=rows)
    lens_s = (offs[1:] - offs[:-1])[keys]
    so = np.zeros(rows + 1, np.int64)
    so[1:] = np.cumsum(lens_s)
    idx = np.repeat(offs[:-1][keys] - so[:-1], lens_s) + np.arange(int(so[-1]), dtype=np.int64)
    out["s"] = dict(values=chars[idx], offsets=so)
    out["i64s"] = dict(values=rng.integers(-2**63, 2**63 - 1, size=rows, dtype=np.int64))
    return out


def c5_columns(p, rows_per_rg, rows_per_page=20000):
    """The nine C5 Column objects of one row group's arrays `p`."""
    rpp_d = _dbp_safe_rows_per_page(rows_per_rg, rows_per_page)
    # Quirk-free by construction: the reference appends each page's
    # whole numValues-long slice to the column store, trailing nils included
    # (Q1, chunk_reader.go:394-397), and from the second row group on decodes a
    # dictionary page into the store's reused backing array, which the first
    # data page's append then overwrites (Q2, chunk_reader.go:235,
    # page_dict.go:50-53).  Both need a chunk with more than one data page, so
    # every column with nulls (lst, oi32) or a dictionary (s) is written the way
    # parquet-go's own writer writes every chunk: ONE data page per chunk
    # (chunk_writer.go:237-246), its level and index streams one bit-packed run
    # each (hybridEncoder.bpEncode, hybrid_encoder.go:59-73).  The columns
    # without nulls keep pyarrow's 20 000 rows per page.
    one = dict(rows_per_page=rows_per_rg, hybrid_groups=REF_HYBRID)
    return [
        Column("lst", DOUBLE, p["lst"]["values"], repetition=LIST, def_levels=p["lst"]["def_levels"],
               rep_levels=p["lst"]["rep_levels"], **one),
        Column("i32", INT32, p["i32"]["values"], rows_per_page=rows_per_page),
        Column("i64d", INT64, p["i64d"]["values"], encoding=DELTA_BINARY_PACKED, rows_per_page=rpp_d),
        Column("f64", DOUBLE, p["f64"]["values"], rows_per_page=rows_per_page),
        Column("f32", FLOAT, p["f32"]["values"], rows_per_page=rows_per_page),
        Column("i96", INT96, p["i96"]["values"], rows_per_page=rows_per_page),
        # the optional int32 column is written with dictionary off (PLAIN)
        Column("oi32", INT32, p["oi32"]["values"], repetition=OPTIONAL, encoding=PLAIN,
               def_levels=p["oi32"]["def_levels"], **one),
        Column("s", BYTE_ARRAY, p["s"]["values"], offsets=p["s"]["offsets"], encoding=RLE_DICTIONARY, **one),
        Column("i64s", INT64, p["i64s"]["values"], codec=SNAPPY, rows_per_page=rows_per_page),
    ]


def config_c5(row_groups=(0,), rows_per_rg=C5_ROWS_PER_RG, seed=5, rows_per_page=20000, as_array=False):
    """C5 row groups `row_groups` (global indices of the 64-row-group file; one
    rank's shard under RG i -> GPU floor(i * G / 64)) written as one file, in
    order, ONE ROW GROUP AT A TIME: a row group's arrays are generated, written
    and dropped before the next (row groups are independent,
    chunk_reader.go:404-431), so a rank holds its file plus one row group's
    arrays, not its whole shard's.  Returns (file bytes, info); as_array: the
    file as a numpy uint8 array (no bytes copy: the bench's multi-GB shard)."""
    rgs = list(row_groups)
    wr = RowGroupWriter()
    for rg in rgs:
        p = c5_row_group_columns(rg, rows_per_rg, seed, rows_per_page)
        cols = c5_columns(p, rows_per_rg, rows_per_page)
        wr.add(cols, rows_per_rg)
        del cols, p
    data = wr.finish()
    if not as_array:
        data = data.tobytes()
    rows = rows_per_rg * len(rgs)

    def part(i):
        """Expected arrays of the file's row group i, regenerated (the same seeds):
        callers hold one row group's arrays at a time."""
        return c5_row_group_columns(rgs[i], rows_per_rg, seed, rows_per_page)

    return data, {"rows": rows, "row_groups": rgs, "rows_per_rg": rows_per_rg, "part": part}
