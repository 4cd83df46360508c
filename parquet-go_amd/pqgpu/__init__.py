"""pqgpu — MI355X (gfx950) Parquet column-chunk decoder behind parquet-go's page-decode surface.

The decode runs in hand-written HIP kernels (parquet-go_amd/csrc, libpqgpu.so);
this package is the host-side binding (ctypes over the C ABI in include/pqgpu.h).
"""
from . import abi  # noqa: F401
from .reader import (DecodedColumn, FileReader, GpuDecoder, ParquetFile, PqgError, chunk_ranges, chunk_span,  # noqa: F401
                     decode_spans, device_job, span_jobs)
