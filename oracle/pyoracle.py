"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of parquet-go's page-decode algorithm
(oracle/pq_oracle.cpp).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module; the product (libpqgpu) never does.
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "parquet-go_amd"))
from pqgpu import abi  # noqa: E402

_lib = None


class StoreRG(C.Structure):
    """pqo_store_rg (include/pqgpu.h)."""
    _fields_ = [("status", C.c_int32), ("value_width", C.c_int32), ("entries", C.c_int64),
                ("values", C.c_void_p), ("nil_flags", C.c_void_p), ("offsets", C.c_void_p),
                ("chars", C.c_int64)]


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle not built: run `make -C oracle`")
        L = C.CDLL(path)
        L.pqo_decode_chunk.argtypes = [C.POINTER(abi.ChunkJob), C.POINTER(abi.ChunkResult),
                                       C.POINTER(abi.PageInfo), C.c_int, C.POINTER(C.c_int)]
        L.pqo_free_result.argtypes = [C.POINTER(abi.ChunkResult)]
        L.pqo_decode_page_range.argtypes = [C.POINTER(abi.ChunkJob), C.c_int, C.c_int, C.POINTER(C.c_int64)]
        L.pqo_decode_page_range.restype = C.c_int64
        L.pqo_unpack8_32.argtypes = [C.c_char_p, C.c_int, C.c_void_p]
        L.pqo_unpack8_64.argtypes = [C.c_char_p, C.c_int, C.c_void_p]
        L.pqo_hybrid_decode.argtypes = [C.c_char_p, C.c_int64, C.c_int, C.c_int64, C.c_void_p]
        L.pqo_snappy_decode.argtypes = [C.c_char_p, C.c_int64, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]
        L.pqo_gzip_decode.argtypes = [C.c_char_p, C.c_int64, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]
        L.pqo_delta_decode64.argtypes = [C.c_char_p, C.c_int64, C.c_int64, C.c_void_p]
        L.pqo_delta_decode32.argtypes = [C.c_char_p, C.c_int64, C.c_int64, C.c_void_p]
        L.pqo_delta_lengths_end.argtypes = [C.c_char_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p]
        L.pqo_assemble.argtypes = [C.POINTER(abi.AssembleArgs)]
        L.pqo_assemble_list.argtypes = [C.POINTER(abi.ListArgs)]
        L.pqo_decode_column_store.argtypes = [C.POINTER(abi.ChunkJob), C.c_int, C.c_int, C.POINTER(StoreRG)]
        L.pqo_free_store.argtypes = [C.POINTER(StoreRG), C.c_int]
        L.pqo_pack_levels.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_void_p]
        L.pqo_go_roundupsize.argtypes = [C.c_int64]
        L.pqo_go_roundupsize.restype = C.c_int64
        _lib = L
    return _lib


def unpack8(data: bytes, width: int, bits: int = 32):
    out = np.zeros(8, dtype=np.int32 if bits == 32 else np.int64)
    fn = lib().pqo_unpack8_32 if bits == 32 else lib().pqo_unpack8_64
    rc = fn(bytes(data) + b"\0" * 8, width, out.ctypes.data)
    assert rc == 0
    return out


def hybrid_decode(buf: bytes, width: int, count: int):
    out = np.zeros(max(count, 1), dtype=np.int32)
    rc = lib().pqo_hybrid_decode(bytes(buf), len(buf), width, count, out.ctypes.data)
    return rc, out[:count]


def snappy_decode(src: bytes, cap: int = 1 << 26):
    dst = np.zeros(max(cap, 1), dtype=np.uint8)
    n = C.c_int64(0)
    rc = lib().pqo_snappy_decode(bytes(src), len(src), dst.ctypes.data, cap, C.byref(n))
    return rc, dst[: n.value].tobytes() if rc == 0 else b""


def gzip_decode(src: bytes, cap: int = 1 << 26):
    dst = np.zeros(max(cap, 1), dtype=np.uint8)
    n = C.c_int64(0)
    rc = lib().pqo_gzip_decode(bytes(src), len(src), dst.ctypes.data, cap, C.byref(n))
    return rc, dst[: n.value].tobytes() if rc == 0 else b""


def delta_decode(buf: bytes, count: int, bits: int = 64):
    out = np.zeros(max(count, 1), dtype=np.int64 if bits == 64 else np.int32)
    fn = lib().pqo_delta_decode64 if bits == 64 else lib().pqo_delta_decode32
    rc = fn(bytes(buf), len(buf), count, out.ctypes.data)
    return rc, out[:count]


def delta_lengths_end(buf: bytes, keep: int):
    """(status, reader end, valuesCount) of a DBP length stream: `keep`
    values decoded one by one, the rest skipped (DeltaBP::skip_rest)."""
    end, cnt = C.c_int64(0), C.c_int64(0)
    rc = lib().pqo_delta_lengths_end(bytes(buf), len(buf), keep, C.byref(end), C.byref(cnt))
    return rc, end.value, cnt.value


class OracleChunk:
    """Host-side decoded chunk from the oracle (numpy copies)."""

    def __init__(self, status, error_page, pages, num_slots, num_values, def_levels, rep_levels,
                 values, offsets, value_width, col_flags=0):
        self.status = status
        self.col_flags = col_flags
        self.error_page = error_page
        self.pages = pages
        self.num_slots = num_slots
        self.num_values = num_values
        self.def_levels = def_levels
        self.rep_levels = rep_levels
        self.values = values
        self.offsets = offsets
        self.value_width = value_width


def decode_chunk(job: abi.ChunkJob, page_cap: int = 1 << 20) -> OracleChunk:
    """Decode one chunk job whose `data` is a HOST pointer."""
    L = lib()
    res = abi.ChunkResult()
    pages = (abi.PageInfo * page_cap)()
    n = C.c_int(0)
    L.pqo_decode_chunk(C.byref(job), C.byref(res), pages, page_cap, C.byref(n))
    plist = [pages[i] for i in range(min(n.value, page_cap))]

    def grab(ptr, nbytes, dtype=np.uint8):
        if not ptr:
            return None
        return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(max(nbytes, 0),)).copy().view(dtype) \
            if nbytes > 0 else np.zeros(0, dtype=dtype)

    out = OracleChunk(res.status, res.error_page, plist, res.num_slots, res.num_values,
                      grab(res.def_levels, res.num_slots), grab(res.rep_levels, res.num_slots),
                      grab(res.values, res.values_bytes),
                      grab(res.offsets, (res.num_values + 1) * 8, np.int64) if res.offsets else None,
                      res.value_width, res.col_flags)
    L.pqo_free_result(C.byref(res))
    return out


def assemble(def_levels, rep_levels, values, max_def, boundary_level, value_width):
    """K8 oracle (ColumnStore.get cursor walk): returns (validity, spaced, offsets, counts)."""
    n = len(def_levels) if def_levels is not None else len(rep_levels)
    d = None if def_levels is None else np.ascontiguousarray(def_levels, dtype=np.uint8)
    r = None if rep_levels is None else np.ascontiguousarray(rep_levels, dtype=np.uint8)
    v = np.ascontiguousarray(values if values is not None else np.zeros(1, np.uint8)).view(np.uint8)
    validity = np.zeros(max((n + 7) // 8, 1), np.uint8)
    spaced = np.zeros(max(n * value_width, 1), np.uint8)
    offsets = np.zeros(n + 1, np.int64)
    a = abi.AssembleArgs()
    a.def_levels = d.ctypes.data if d is not None else None
    a.rep_levels = r.ctypes.data if r is not None else None
    a.values = v.ctypes.data
    a.num_slots, a.max_def, a.boundary_level, a.value_width = n, max_def, boundary_level, value_width
    a.validity, a.values_spaced, a.offsets = validity.ctypes.data, spaced.ctypes.data if value_width else None, \
        offsets.ctypes.data
    rc = lib().pqo_assemble(C.byref(a))
    assert rc == 0
    return (validity[:(n + 7) // 8], spaced[:n * value_width], offsets[:a.num_boundaries + 1],
            (a.num_valid, a.null_count, a.num_boundaries))


def assemble_list(def_levels, rep_levels, values, max_def, list_def, elem_def, value_width):
    """K8 list export oracle: returns (list_validity, list_offsets, elem_validity,
    elem_values, (rows, elements, valid, null_lists)); bitmaps trimmed to their bits."""
    n = len(def_levels)
    d = np.ascontiguousarray(def_levels, dtype=np.uint8)
    r = None if rep_levels is None else np.ascontiguousarray(rep_levels, dtype=np.uint8)
    v = np.ascontiguousarray(values if values is not None else np.zeros(1, np.uint8)).view(np.uint8)
    lv = np.zeros(max((n + 7) // 8, 1), np.uint8)
    ev = np.zeros(max((n + 7) // 8, 1), np.uint8)
    lo = np.zeros(n + 1, np.int32)
    evals = np.zeros(max(n * value_width, 1), np.uint8)
    a = abi.ListArgs()
    a.def_levels = d.ctypes.data
    a.rep_levels = r.ctypes.data if r is not None else None
    a.values = v.ctypes.data
    a.num_slots, a.max_def, a.list_def, a.elem_def, a.value_width = n, max_def, list_def, elem_def, value_width
    a.list_validity, a.list_offsets, a.elem_validity = lv.ctypes.data, lo.ctypes.data, ev.ctypes.data
    a.elem_values = evals.ctypes.data if value_width else None
    rc = lib().pqo_assemble_list(C.byref(a))
    assert rc == 0, rc
    rows, el = a.num_rows, a.num_elements
    return (lv[:(rows + 7) // 8], lo[:rows + 1], ev[:(el + 7) // 8], evals[:el * value_width],
            (rows, el, a.num_valid, a.null_lists))


def decode_column_store(jobs, quirks):
    """The reference's ColumnStore.values contents per row group (Q1/Q2 triage):
    list of (status, values, nil flags u8) where values are the entries' bytes
    (entries x width) for fixed-width columns and (chars, offsets[entries + 1])
    for byte arrays."""
    n = len(jobs)
    arr = (abi.ChunkJob * max(n, 1))(*jobs)
    out = (StoreRG * max(n, 1))()
    rc = lib().pqo_decode_column_store(arr, n, quirks, out)
    assert rc == 0, rc
    res = []
    for i in range(n):
        o = out[i]
        if o.status != 0:
            res.append((o.status, None, None))
            continue
        cnt = o.entries
        nil = np.ctypeslib.as_array(C.cast(o.nil_flags, C.POINTER(C.c_uint8)), shape=(max(cnt, 1),))[:cnt].copy()
        if o.value_width > 0:
            vals = np.ctypeslib.as_array(C.cast(o.values, C.POINTER(C.c_uint8)),
                                         shape=(max(cnt * o.value_width, 1),))[:cnt * o.value_width].copy()
        else:
            chars = np.ctypeslib.as_array(C.cast(o.values, C.POINTER(C.c_uint8)), shape=(max(o.chars, 1),))
            offs = np.ctypeslib.as_array(C.cast(o.offsets, C.POINTER(C.c_int64)), shape=(cnt + 1,))
            vals = (chars[:o.chars].copy(), offs.copy())
        res.append((0, vals, nil))
    lib().pqo_free_store(out, n)
    return res


def pack_levels(levels, max_level):
    """packedArray bytes of `levels` (packed_array.go:34-101)."""
    lv = np.ascontiguousarray(levels, dtype=np.uint8)
    bw = int(max_level).bit_length()
    out = np.zeros(max((len(lv) + 7) // 8 * bw, 1), np.uint8)
    rc = lib().pqo_pack_levels(lv.ctypes.data if len(lv) else None, len(lv), max_level, out.ctypes.data)
    assert rc == 0
    return out[:(len(lv) + 7) // 8 * bw]
