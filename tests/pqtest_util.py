"""Shared helpers for the parity tests: hand-built pages, chunk jobs, pyarrow expectations."""
import ctypes as C
import io
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "parquet-go_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

from pqgpu import abi  # noqa: E402


# ---------------------------------------------------------------- thrift compact writer (tests)
def uvarint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def zigzag(v):
    return uvarint((v << 1) ^ (v >> 63) if v < 0 else v << 1)


class TW:
    def __init__(self):
        self.b = bytearray()
        self.last = [0]

    def field(self, fid, ctype):
        d = fid - self.last[-1]
        if 0 < d <= 15:
            self.b.append((d << 4) | ctype)
        else:
            self.b.append(ctype)
            self.b += zigzag(fid)
        self.last[-1] = fid

    def i32(self, fid, v):
        self.field(fid, 5)
        self.b += zigzag(v)
        return self

    def i64(self, fid, v):
        self.field(fid, 6)
        self.b += zigzag(v)
        return self

    def boolean(self, fid, v):
        self.field(fid, 1 if v else 2)
        return self

    def begin(self, fid):
        self.field(fid, 12)
        self.last.append(0)
        return self

    def end(self):
        self.b.append(0)
        self.last.pop()
        return self

    def stop(self):
        self.b.append(0)
        return bytes(self.b)


def page_header_v1(usize, csize, nvals, enc, def_enc=3, rep_enc=3):
    t = TW()
    t.i32(1, 0).i32(2, usize).i32(3, csize)
    t.begin(5).i32(1, nvals).i32(2, enc).i32(3, def_enc).i32(4, rep_enc).end()
    return t.stop()


def page_header_dict(usize, csize, nvals, enc=0):
    t = TW()
    t.i32(1, 2).i32(2, usize).i32(3, csize)
    t.begin(7).i32(1, nvals).i32(2, enc).end()
    return t.stop()


def page_header_v2(usize, csize, nvals, nnulls, nrows, enc, def_len, rep_len, is_comp=True):
    t = TW()
    t.i32(1, 3).i32(2, usize).i32(3, csize)
    t.begin(8).i32(1, nvals).i32(2, nnulls).i32(3, nrows).i32(4, enc).i32(5, def_len).i32(6, rep_len)
    t.boolean(7, is_comp).end()
    return t.stop()


def u32(v):
    return int(v).to_bytes(4, "little")


def v1_page(values: bytes, nvals, enc, rep: bytes = None, defs: bytes = None):
    body = b""
    if rep is not None:
        body += u32(len(rep)) + rep
    if defs is not None:
        body += u32(len(defs)) + defs
    body += values
    return page_header_v1(len(body), len(body), nvals, enc) + body


def chunk_job(chunk: bytes, ptype, max_def=0, max_rep=0, codec=0, type_length=-1, data_page_offset=0,
              has_dict_off=False, keep=None):
    """Host chunk job over `chunk` (keep a reference to the buffer in `keep`)."""
    buf = np.frombuffer(chunk, dtype=np.uint8).copy() if len(chunk) else np.zeros(1, np.uint8)
    if keep is not None:
        keep.append(buf)
    j = abi.ChunkJob()
    j.col.physical_type = ptype
    j.col.type_length = type_length
    j.col.max_def = max_def
    j.col.max_rep = max_rep
    j.col.codec = codec
    j.data = buf.ctypes.data
    j.data_len = len(chunk)
    j.total_compressed_size = len(chunk)
    j.data_page_offset = data_page_offset
    j.num_values_hint = 0
    j.total_uncompressed_size = len(chunk)
    j.has_dict_page_offset = int(has_dict_off)
    return j, buf


def arrow_column(data: bytes, col=0):
    import pyarrow.parquet as pq
    t = pq.read_table(io.BytesIO(data))
    return t.column(col)


def dense_values(arrow_col, np_dtype):
    """Non-null values of an arrow column as a numpy array."""
    a = arrow_col.combine_chunks()
    vals = a.drop_null() if hasattr(a, "drop_null") else a.filter(a.is_valid())
    return np.asarray(vals.to_numpy(zero_copy_only=False)).astype(np_dtype)
