"""Host-side mirror of parquet-go's reader surface over libpqgpu.

parquet-go (fraugster/parquet-go v0.2.1) reads a file with
    NewFileReader(r, columns...)      file_reader.go:27-48
    FileReader.readRowGroup / PreLoad file_reader.go:51-98  → readRowGroup chunk_reader.go:404-431
and decodes each selected column chunk with readChunk → readPages →
readPageData (chunk_reader.go:206-402).  This module keeps those names and
meanings; the page decode itself runs in the HIP kernels of libpqgpu.
Column projection follows schema.isSelected (schema.go:296-312): an empty
selection reads every column.
"""
import ctypes as C
import os

import numpy as np

from . import abi
from ._lib import lib


class PqgError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = int(code)
        super().__init__("%s: %s (%d)" % (what, abi.status_name(code), code))


def _check(rc, what):
    if rc != 0:
        raise PqgError(rc, what)


class ParquetFile:
    """Footer + schema of a parquet file (readFileMetaData file_meta.go:14-62).

    ParquetFile(data) holds the whole file in host memory; ParquetFile.open(path)
    reads only the first 4 bytes and the footer, and chunk bytes are fetched by
    byte range on demand (read_range), as readChunk seeks to each chunk
    (chunk_reader.go:332-340)."""

    def __init__(self, data=None, *, _path=None):
        L = lib()
        h = C.c_void_p()
        self.path = _path
        if _path is None:
            if isinstance(data, np.ndarray) and data.dtype == np.uint8 and data.ndim == 1 and data.flags.c_contiguous:
                self.data = data  # a large file (the bench's C5 shard): no second copy
                self._buf = data
            else:
                self.data = bytes(data)
                self._buf = np.frombuffer(self.data, dtype=np.uint8)
            self.size = len(self.data)
            ptr = self._buf.ctypes.data if self.size else None
            _check(L.pqg_file_open(C.cast(ptr, C.c_char_p) if ptr else b"", self.size, C.byref(h)), "pqg_file_open")
        else:
            self.data = None
            self._buf = None
            self.size = os.path.getsize(_path)
            with open(_path, "rb") as f:
                head = f.read(4)
                f.seek(max(0, self.size - 8))
                last8 = f.read(8)
                fl = int.from_bytes(last8[:4], "little", signed=True) if len(last8) == 8 else 0
                n = min(self.size, max(fl, 0) + 8)
                f.seek(self.size - n)
                tail = f.read(n)
            _check(L.pqg_file_open_tail(head, len(head), tail, len(tail), self.size, C.byref(h)), "pqg_file_open_tail")
        self._h = h
        self.num_columns = L.pqg_file_num_columns(h)
        self.num_row_groups = L.pqg_file_num_row_groups(h)
        self.num_rows = L.pqg_file_num_rows(h)
        self.columns = []
        for i in range(self.num_columns):
            ci = abi.ColumnInfo()
            _check(L.pqg_file_column(h, i, C.byref(ci)), "pqg_file_column")
            self.columns.append(ci)
        self.schema_nodes = []  # depth first, below the root (pqg_file_schema_node)
        for i in range(L.pqg_file_num_schema_nodes(h)):
            sn = abi.SchemaNode()
            _check(L.pqg_file_schema_node(h, i, C.byref(sn)), "pqg_file_schema_node")
            self.schema_nodes.append(sn)

    @classmethod
    def open(cls, path):
        return cls(_path=path)

    def read_range(self, lo, hi):
        """Bytes [lo, hi) of the file (shorter at its end)."""
        lo, hi = max(0, lo), min(hi, self.size)
        if hi <= lo:
            return np.zeros(0, np.uint8)
        if self.path is None:
            return self._buf[lo:hi]
        fd = os.open(self.path, os.O_RDONLY)
        try:
            return np.frombuffer(os.pread(fd, hi - lo, lo), dtype=np.uint8)
        finally:
            os.close(fd)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().pqg_file_close(h)
            self._h = None

    def column_index(self, path):
        for i, c in enumerate(self.columns):
            if c.path.decode() == path:
                return i
        raise KeyError(path)

    def row_group_rows(self, rg):
        return lib().pqg_file_row_group_rows(self._h, rg)

    def chunk_meta(self, rg, col):
        m = abi.ChunkMeta()
        _check(lib().pqg_file_chunk(self._h, rg, col, C.byref(m)), "pqg_file_chunk")
        return m

    def host_job(self, rg, col):
        """A chunk job whose data pointer is HOST memory (for the CPU oracle)."""
        m = self.chunk_meta(rg, col)
        job = abi.ChunkJob()
        job.col = self.columns[col].desc
        job.col.codec = m.codec
        start = max(0, min(m.start, self.size))
        if self.path is None:
            job.data = self._buf.ctypes.data + start
            job.data_len = self.size - start
        else:  # the chunk's own bytes, kept alive by the job (not the file)
            b = np.ascontiguousarray(self.read_range(start, start + m.total_compressed_size))
            job._keep = b
            job.data = b.ctypes.data if b.nbytes else None
            job.data_len = b.nbytes
        job.total_compressed_size = m.total_compressed_size
        job.data_page_offset = m.data_page_offset - m.start
        job.num_values_hint = m.num_values
        job.total_uncompressed_size = m.total_uncompressed_size
        job.has_dict_page_offset = m.has_dict_page_offset
        return job, m


class DecodedColumn:
    """Decoded chunk on the host: def/rep levels + dense values[:nn] (readValues outputs)."""

    def __init__(self, status, error_page, num_slots, num_values, value_width, def_levels, rep_levels, values,
                 pages, offsets=None):
        self.status = status
        self.error_page = error_page
        self.num_slots = num_slots
        self.num_values = num_values
        self.value_width = value_width
        self.def_levels = def_levels
        self.rep_levels = rep_levels
        self.values = values          # fixed width: dense values; variable length: chars
        self.offsets = offsets        # variable length: int64[num_values + 1]
        self.pages = pages


class GpuDecoder:
    """One decode context per GPU (pqg_ctx)."""

    def __init__(self, device=0):
        self.L = lib()
        h = C.c_void_p()
        _check(self.L.pqg_ctx_create(device, C.byref(h)), "pqg_ctx_create")
        self.ctx = h
        self._bufs = []

    def close(self):
        for p in self._bufs:
            self.L.pqg_device_free(self.ctx, p)
        self._bufs = []
        if self.ctx:
            self.L.pqg_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- device memory
    def upload(self, data):
        arr = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        p = C.c_void_p()
        _check(self.L.pqg_device_alloc(self.ctx, max(arr.nbytes, 1), C.byref(p)), "pqg_device_alloc")
        if arr.nbytes:
            _check(self.L.pqg_memcpy_h2d(self.ctx, p, arr.ctypes.data, arr.nbytes), "pqg_memcpy_h2d")
        self._bufs.append(p)
        return p.value

    def upload_ranges(self, buf, ranges):
        """One device buffer holding buf[lo:hi] for each (lo, hi) of `ranges`,
        packed in order, copied range by range (no packed host copy)."""
        total = sum(hi - lo for lo, hi in ranges)
        p = C.c_void_p()
        _check(self.L.pqg_device_alloc(self.ctx, max(total, 1), C.byref(p)), "pqg_device_alloc")
        self._bufs.append(p)
        at = 0
        for lo, hi in ranges:
            if hi > lo:
                src = buf[lo:hi]
                _check(self.L.pqg_memcpy_h2d(self.ctx, C.c_void_p(p.value + at), src.ctypes.data, hi - lo),
                       "pqg_memcpy_h2d")
            at += hi - lo
        return p.value

    def free(self, ptr):
        for i, p in enumerate(self._bufs):
            if p.value == ptr:
                self.L.pqg_device_free(self.ctx, p)
                del self._bufs[i]
                return

    def d2h(self, ptr, nbytes, dtype=np.uint8):
        out = np.empty(max(nbytes, 0), dtype=np.uint8)
        if nbytes > 0:
            _check(self.L.pqg_memcpy_d2h(self.ctx, out.ctypes.data, C.c_void_p(ptr), nbytes), "pqg_memcpy_d2h")
        return out.view(dtype) if dtype != np.uint8 else out

    # ---- decode
    def decode_jobs(self, jobs):
        n = len(jobs)
        arr = (abi.ChunkJob * max(n, 1))(*jobs)
        res = (abi.ChunkResult * max(n, 1))()
        _check(self.L.pqg_decode_chunks(self.ctx, arr, n, res), "pqg_decode_chunks")
        return [res[i] for i in range(n)]

    def pages(self, job_index, cap=1 << 20):
        buf = (abi.PageInfo * cap)()
        k = self.L.pqg_get_pages(self.ctx, job_index, buf, cap)
        if k < 0:
            raise PqgError(k, "pqg_get_pages")
        return [buf[i] for i in range(k)]

    def debug_job(self, job_index):
        """(serial_walk, candidates, pages, scratch_bytes, pipeline_launches) of the last decode."""
        out = (C.c_int64 * 5)()
        k = self.L.pqg_debug_job(self.ctx, job_index, out, 5)
        if k < 0:
            raise PqgError(k, "pqg_debug_job")
        return tuple(int(out[i]) for i in range(k))

    def timings(self):
        out = (C.c_float * 16)()
        k = self.L.pqg_last_timings(self.ctx, out, 16)
        return [out[i] for i in range(max(k, 0))]

    def assemble(self, def_ptr, rep_ptr, values_ptr, num_slots, max_def, boundary_level=0, value_width=0,
                 validity=True, spaced=False, offsets=True):
        """K8 on device arrays (e.g. a ChunkResult's levels/values): allocates the
        requested outputs and returns (AssembleArgs, validity_ptr, spaced_ptr,
        offsets_ptr).  Mirrors ColumnStore.get (data_store.go:158-203)."""
        a = abi.AssembleArgs()
        a.def_levels, a.rep_levels, a.values = def_ptr or None, rep_ptr or None, values_ptr or None
        a.num_slots, a.max_def, a.boundary_level, a.value_width = num_slots, max_def, boundary_level, value_width

        def alloc(nbytes):
            p = C.c_void_p()
            _check(self.L.pqg_device_alloc(self.ctx, max(nbytes, 1), C.byref(p)), "pqg_device_alloc")
            self._bufs.append(p)
            return p.value

        vp = alloc((num_slots + 7) // 8) if validity else None
        sp = alloc(num_slots * value_width) if spaced else None
        op = alloc((num_slots + 1) * 8) if offsets else None
        a.validity, a.values_spaced, a.offsets = vp, sp, op
        _check(self.L.pqg_assemble(self.ctx, C.byref(a)), "pqg_assemble")
        return a, vp, sp, op

    def assemble_list(self, def_ptr, rep_ptr, values_ptr, num_slots, max_def, list_def=1, elem_def=2,
                      value_width=0, values=True):
        """K8 list export (Arrow LIST layout) of device level/value arrays.
        Returns (ListArgs, list_validity, list_offsets, elem_validity, elem_values)
        device pointers (elem_values None unless `values`)."""
        a = abi.ListArgs()
        a.def_levels, a.rep_levels, a.values = def_ptr, rep_ptr or None, values_ptr or None
        a.num_slots, a.max_def, a.list_def, a.elem_def = num_slots, max_def, list_def, elem_def
        a.value_width = value_width

        def alloc(nbytes):
            p = C.c_void_p()
            _check(self.L.pqg_device_alloc(self.ctx, max(nbytes, 1), C.byref(p)), "pqg_device_alloc")
            self._bufs.append(p)
            return p.value

        bm = (num_slots + 31) // 32 * 4
        a.list_validity, a.list_offsets, a.elem_validity = alloc(bm), alloc((num_slots + 1) * 4), alloc(bm)
        a.elem_values = alloc(num_slots * value_width) if values and value_width else None
        _check(self.L.pqg_assemble_list(self.ctx, C.byref(a)), "pqg_assemble_list")
        return a, a.list_validity, a.list_offsets, a.elem_validity, a.elem_values

    def download(self, r, job_index=None):
        lv_def = self.d2h(r.def_levels, r.num_slots) if (r.def_levels and r.status == 0) else None
        lv_rep = self.d2h(r.rep_levels, r.num_slots) if (r.rep_levels and r.status == 0) else None
        vals = self.d2h(r.values, r.values_bytes) if r.status == 0 else None
        offs = self.d2h(r.offsets, (r.num_values + 1) * 8, np.int64) if (r.offsets and r.status == 0) else None
        pages = self.pages(job_index) if job_index is not None else None
        return DecodedColumn(r.status, r.error_page, r.num_slots, r.num_values, r.value_width, lv_def, lv_rep,
                             vals, pages, offs)


def device_job(pf: ParquetFile, rg, col, dev_ptr_of_file):
    """Chunk job pointing into a device copy of the whole file."""
    job, m = pf.host_job(rg, col)
    start = max(0, min(m.start, len(pf.data)))
    job.data = dev_ptr_of_file + start
    return job


def chunk_span(pf: ParquetFile, specs):
    """The byte span [lo, hi) covering the chunks of (rg, col) pairs
    ([start, start + TotalCompressedSize) each, chunk_reader.go:332-340) and
    their ChunkMetas."""
    metas = [pf.chunk_meta(rg, c) for rg, c in specs]
    lo = min(m.start for m in metas)
    hi = max(m.start + m.total_compressed_size for m in metas)
    return max(0, lo), min(hi, pf.size), metas


def chunk_ranges(pf: ParquetFile, specs, to_eof=()):
    """The byte ranges the chunks of (rg, col) pairs occupy ([start, start +
    TotalCompressedSize) each, clipped to the file; [start, end of file) for the
    spec indices in `to_eof`), sorted, with overlapping or adjacent ranges
    merged: [(lo, hi)], and the chunks' ChunkMetas."""
    metas = [pf.chunk_meta(rg, c) for rg, c in specs]
    rs = sorted((max(0, min(m.start, pf.size)),
                 pf.size if i in to_eof else max(0, min(m.start + m.total_compressed_size, pf.size)))
                for i, m in enumerate(metas))
    out = []
    for lo, hi in rs:
        if out and lo <= out[-1][1]:
            out[-1][1] = max(out[-1][1], hi)
        else:
            out.append([lo, hi])
    return [tuple(r) for r in out], metas


def span_jobs(pf: ParquetFile, specs, dec, to_eof=()):
    """Chunk jobs for (rg, col) pairs with only their chunks' bytes uploaded,
    packed into one device buffer (merged ranges, chunk_ranges), each job
    pointing into it.  Unselected chunks are never read, as skipChunk seeks past
    them (chunk_reader.go:286-312).  A job's readable bytes run to the end of
    its merged range.  That range holds every page HEADER readPages reads (it
    reads headers while TotalCompressedSize - Count() > 0, chunk_reader.go:212-
    217), but the reference then reads the whole page from the file, so a last
    page overrunning an understated TotalCompressedSize needs bytes past it:
    decode_spans re-uploads such chunks to the end of the file (`to_eof`).
    Returns (jobs, device pointer, bytes uploaded)."""
    ranges, metas = chunk_ranges(pf, specs, to_eof)
    total = sum(hi - lo for lo, hi in ranges)
    base = []  # packed offset of each range
    at = 0
    for lo, hi in ranges:
        base.append(at)
        at += hi - lo
    if pf._buf is not None:  # the file in host memory: each range straight from it
        dev = dec.upload_ranges(pf._buf, ranges)
    else:
        host = np.empty(max(total, 1), dtype=np.uint8)
        for (lo, hi), b in zip(ranges, base):
            host[b:b + hi - lo] = pf.read_range(lo, hi)
        dev = dec.upload(host)
        del host
    jobs = []
    for (rg, c), m in zip(specs, metas):
        job = abi.ChunkJob()
        job.col = pf.columns[c].desc
        job.col.codec = m.codec
        job.total_compressed_size = m.total_compressed_size
        job.data_page_offset = m.data_page_offset - m.start
        job.num_values_hint = m.num_values
        job.total_uncompressed_size = m.total_uncompressed_size
        job.has_dict_page_offset = m.has_dict_page_offset
        start = max(0, min(m.start, pf.size))
        k = max(i for i, (lo, _) in enumerate(ranges) if lo <= start)
        lo, hi = ranges[k]
        job.data = dev + base[k] + (start - lo)
        job.data_len = hi - start
        jobs.append(job)
    return jobs, dev, total


def decode_spans(pf: ParquetFile, specs, dec):
    """span_jobs + pqg_decode_chunks for (rg, col) pairs.  A chunk whose decode
    ends in EOF / size mismatch while the file holds bytes past its uploaded
    range (a page overrunning TotalCompressedSize, which the reference still
    reads whole: chunk_reader.go:212-280) is decoded again with the bytes to the
    end of the file, in a second batched call (device outputs are only valid
    until the next decode on `dec`).  Returns (results, device buffer, bytes
    uploaded); the caller frees the buffer after using the outputs."""
    jobs, dev, nbytes = span_jobs(pf, specs, dec)
    res = dec.decode_jobs(jobs)
    retry = set()
    for i, (job, r) in enumerate(zip(jobs, res)):
        m = pf.chunk_meta(*specs[i])
        start = max(0, min(m.start, pf.size))
        if r.status in (abi.STATUS_CODES["EOF"], abi.STATUS_CODES["SIZE"]) and job.data_len < pf.size - start:
            retry.add(i)
    if retry:
        dec.free(dev)
        jobs, dev, nb2 = span_jobs(pf, specs, dec, to_eof=retry)
        nbytes += nb2
        res = dec.decode_jobs(jobs)
    return res, dev, nbytes


class FileReader:
    """Mirror of parquet-go's FileReader (file_reader.go:27-118): the selected
    columns of a file (dotted paths, schema.isSelected schema.go:296-312; none =
    all), decoded one row group at a time on the GPU.  `source` is the file's
    bytes or a path (then only the footer and the selected chunks are read);
    each row group uploads only its selected chunks' bytes (span_jobs)."""

    def __init__(self, source, *columns, device=0, decoder=None):
        self.file = ParquetFile.open(source) if isinstance(source, (str, os.PathLike)) else ParquetFile(source)
        self.dec = decoder or GpuDecoder(device)
        self.selected = self._select(columns)
        self.row_group_position = 0
        self.uploaded_bytes = 0   # H2D bytes so far (projection pushdown check)
        self._rows = None         # NextRow state (pqgpu.rows.RowReader)

    def _select(self, columns):
        if not columns:
            return list(range(self.file.num_columns))
        out = []
        for i, c in enumerate(self.file.columns):
            path = c.path.decode()
            if any(path == p or path.startswith(p + ".") for p in columns):
                out.append(i)
        return out

    def row_group_count(self):
        return self.file.num_row_groups

    def num_rows(self):
        return self.file.num_rows

    def decode_row_groups(self, rgs):
        """readRowGroup (chunk_reader.go:404-431) for the selected columns of
        every row group in `rgs`, one batched decode: [(rg, col, ChunkResult)]
        with device outputs (valid until the next decode on the decoder)."""
        specs = [(rg, c) for rg in rgs for c in self.selected]
        if not specs:
            return []
        res, dev, nbytes = decode_spans(self.file, specs, self.dec)
        self.uploaded_bytes += nbytes
        self.dec.free(dev)
        return [(rg, c, r) for (rg, c), r in zip(specs, res)]

    def read_row_group(self, rg):
        """One row group's selected columns, downloaded: {path: DecodedColumn}."""
        specs = [(rg, c) for c in self.selected]
        if not specs:
            return {}
        res, dev, nbytes = decode_spans(self.file, specs, self.dec)
        self.uploaded_bytes += nbytes
        try:
            return {self.file.columns[c].path.decode(): self.dec.download(r, i)
                    for i, ((_, c), r) in enumerate(zip(specs, res))}
        finally:
            self.dec.free(dev)

    def next_row(self):
        """NextRow (file_reader.go:101-108): the next row of the selected
        columns as a dict (pqgpu.rows), decoding the next row group on the GPU
        when the current one is used up; EOFError after the last row."""
        if self._rows is None:
            from .rows import RowReader
            self._rows = RowReader(self.file, self.selected, self._decode_for_rows)
        return self._rows.next_row()

    def _decode_for_rows(self, rg):
        specs = [(rg, c) for c in self.selected]
        if not specs:
            return {}
        res, dev, nbytes = decode_spans(self.file, specs, self.dec)
        self.uploaded_bytes += nbytes
        try:
            return {c: self.dec.download(r, i) for i, ((_, c), r) in enumerate(zip(specs, res))}
        finally:
            self.dec.free(dev)

    def close(self):
        pass
