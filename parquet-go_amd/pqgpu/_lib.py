"""Loader for libpqgpu.so (the HIP product library, built in-tree)."""
import ctypes as C
import os

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(HERE), "csrc", "libpqgpu.so")
# diagnostics only: PQG_LIB may name the -DPQG_PROFILE build (libpqgpu_prof.so)
LIB_PATH = os.environ.get("PQG_LIB") or LIB_PATH

_lib = None


def lib():
    """Load libpqgpu.so; raise loudly if it has not been built (no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libpqgpu.so not built (%s): run __graft_entry__.build() or make -C parquet-go_amd/csrc"
                           % LIB_PATH)
    L = C.CDLL(LIB_PATH)
    P, I, I64 = C.c_void_p, C.c_int, C.c_int64
    sig = {
        "pqg_ctx_create": ([I, C.POINTER(P)], I),
        "pqg_ctx_destroy": ([P], None),
        "pqg_status_string": ([I], C.c_char_p),
        "pqg_device_alloc": ([P, I64, C.POINTER(P)], I),
        "pqg_device_free": ([P, P], I),
        "pqg_memcpy_h2d": ([P, P, P, I64], I),
        "pqg_memcpy_d2h": ([P, P, P, I64], I),
        "pqg_decode_chunks_async": ([P, C.POINTER(abi.ChunkJob), I], I),
        "pqg_sync": ([P, C.POINTER(abi.ChunkResult), I], I),
        "pqg_decode_chunks": ([P, C.POINTER(abi.ChunkJob), I, C.POINTER(abi.ChunkResult)], I),
        "pqg_get_pages": ([P, I, C.POINTER(abi.PageInfo), I], I),
        "pqg_last_timings": ([P, C.POINTER(C.c_float), I], I),
        "pqg_set_timing": ([P, I], I),
        "pqg_debug_job": ([P, I, C.POINTER(I64), I], I),
        "pqg_debug_counters": ([P, C.POINTER(C.c_uint64), I], I),
        "pqg_bench_decode": ([P, C.POINTER(abi.ChunkJob), I, I, C.POINTER(C.c_float), C.POINTER(C.c_float), I], I),
        "pqg_assemble": ([P, C.POINTER(abi.AssembleArgs)], I),
        "pqg_assemble_list": ([P, C.POINTER(abi.ListArgs)], I),
        "pqg_last_assemble_ms": ([P, C.POINTER(C.c_float)], I),
        "pqg_decode_page": ([P, C.POINTER(abi.PageJob), C.POINTER(abi.ChunkResult)], I),
        "pqg_block_decompress": ([P, I, C.c_char_p, I64, P, I64, C.POINTER(I64)], I),
        "pqg_pack_levels": ([P, P, I64, I, P], I),
        "pqg_file_open": ([C.c_char_p, I64, C.POINTER(P)], I),
        "pqg_file_open_tail": ([C.c_char_p, I64, C.c_char_p, I64, I64, C.POINTER(P)], I),
        "pqg_file_close": ([P], None),
        "pqg_file_num_columns": ([P], I),
        "pqg_file_num_row_groups": ([P], I),
        "pqg_file_num_rows": ([P], I64),
        "pqg_file_row_group_rows": ([P, I], I64),
        "pqg_file_column": ([P, I, C.POINTER(abi.ColumnInfo)], I),
        "pqg_file_chunk": ([P, I, I, C.POINTER(abi.ChunkMeta)], I),
        "pqg_file_num_schema_nodes": ([P], I),
        "pqg_file_schema_node": ([P, I, C.POINTER(abi.SchemaNode)], I),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


EXPORTED = [
    "pqg_ctx_create", "pqg_ctx_destroy", "pqg_status_string", "pqg_device_alloc", "pqg_device_free",
    "pqg_memcpy_h2d", "pqg_memcpy_d2h", "pqg_decode_chunks_async", "pqg_sync", "pqg_decode_chunks",
    "pqg_get_pages", "pqg_last_timings", "pqg_set_timing", "pqg_debug_job", "pqg_debug_counters", "pqg_bench_decode", "pqg_assemble",
    "pqg_assemble_list", "pqg_last_assemble_ms", "pqg_decode_page", "pqg_block_decompress", "pqg_pack_levels", "pqg_file_open", "pqg_file_open_tail",
    "pqg_file_close",
    "pqg_file_num_columns", "pqg_file_num_row_groups", "pqg_file_num_rows", "pqg_file_row_group_rows",
    "pqg_file_column", "pqg_file_chunk", "pqg_file_num_schema_nodes", "pqg_file_schema_node",
]
