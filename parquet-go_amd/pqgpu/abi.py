"""ctypes mirror of include/pqgpu.h (the C ABI of libpqgpu).

Only plain structs and enums live here; no library is loaded by this module.
"""
import ctypes as C

# parquet.thrift enums
BOOLEAN, INT32, INT64, INT96, FLOAT, DOUBLE, BYTE_ARRAY, FIXED_LEN_BYTE_ARRAY = range(8)
ENC_PLAIN = 0
ENC_PLAIN_DICTIONARY = 2
ENC_RLE = 3
ENC_BIT_PACKED = 4
ENC_DELTA_BINARY_PACKED = 5
ENC_DELTA_LENGTH_BYTE_ARRAY = 6
ENC_DELTA_BYTE_ARRAY = 7
ENC_RLE_DICTIONARY = 8
CODEC_UNCOMPRESSED, CODEC_SNAPPY, CODEC_GZIP = 0, 1, 2
PAGE_DATA, PAGE_INDEX, PAGE_DICTIONARY, PAGE_DATA_V2 = 0, 1, 2, 3

STATUS = {
    0: "OK",
    -1: "EOF",
    -2: "THRIFT",
    -3: "PAGE_HEADER",
    -4: "SIZE",
    -5: "SNAPPY",
    -6: "RLE",
    -7: "DICT_INDEX",
    -8: "BIT_WIDTH",
    -9: "DELTA",
    -10: "UNSUPPORTED",
    -11: "DICT_PAGE",
    -12: "BYTE_ARRAY",
    -13: "LEVELS",
    -14: "FIXED_LEN",
    -15: "GZIP",
    -20: "CAPACITY",
    -21: "INVALID_ARG",
    -22: "HIP",
    -23: "METADATA",
    -24: "NOT_BUILT",
}
OK = 0
ERR_CAPACITY = -20
STATUS_CODES = {v: k for k, v in STATUS.items()}

FIXED_WIDTH = {BOOLEAN: 1, INT32: 4, INT64: 8, INT96: 12, FLOAT: 4, DOUBLE: 8}


class ColumnDesc(C.Structure):
    _fields_ = [
        ("physical_type", C.c_int32),
        ("type_length", C.c_int32),
        ("max_def", C.c_int32),
        ("max_rep", C.c_int32),
        ("codec", C.c_int32),
        ("flags", C.c_int32),
    ]


class ChunkJob(C.Structure):
    _fields_ = [
        ("col", ColumnDesc),
        ("data", C.c_void_p),
        ("data_len", C.c_int64),
        ("total_compressed_size", C.c_int64),
        ("data_page_offset", C.c_int64),
        ("num_values_hint", C.c_int64),
        ("total_uncompressed_size", C.c_int64),
        ("has_dict_page_offset", C.c_int32),
        ("quirks", C.c_int32),
    ]


QUIRK_Q1_PAGE_NILS, QUIRK_Q2_DICT_ALIAS = 1, 2


class PageJob(C.Structure):
    """pqg_page_job (include/pqgpu.h)."""
    _fields_ = [("col", ColumnDesc), ("page", C.c_void_p), ("page_len", C.c_int64), ("dict_page", C.c_void_p),
                ("dict_page_len", C.c_int64)]


class ChunkResult(C.Structure):
    _fields_ = [
        ("status", C.c_int32),
        ("error_page", C.c_int32),
        ("num_pages", C.c_int32),
        ("value_width", C.c_int32),
        ("col_flags", C.c_int32),
        ("reserved", C.c_int32),
        ("num_slots", C.c_int64),
        ("num_values", C.c_int64),
        ("values_bytes", C.c_int64),
        ("def_levels", C.c_void_p),
        ("rep_levels", C.c_void_p),
        ("values", C.c_void_p),
        ("offsets", C.c_void_p),
    ]


class PageInfo(C.Structure):
    _fields_ = [
        ("header_offset", C.c_int64),
        ("payload_offset", C.c_int64),
        ("slot_offset", C.c_int64),
        ("value_offset", C.c_int64),
        ("page_type", C.c_int32),
        ("encoding", C.c_int32),
        ("num_values", C.c_int32),
        ("not_null", C.c_int32),
        ("compressed_size", C.c_int32),
        ("uncompressed_size", C.c_int32),
        ("def_len", C.c_int32),
        ("rep_len", C.c_int32),
        ("def_encoding", C.c_int32),
        ("rep_encoding", C.c_int32),
        ("status", C.c_int32),
        ("flags", C.c_int32),
    ]


class ColumnInfo(C.Structure):
    _fields_ = [("desc", ColumnDesc), ("path", C.c_char * 256)]


class SchemaNode(C.Structure):
    _fields_ = [("name", C.c_char * 128), ("repetition", C.c_int32), ("num_children", C.c_int32),
                ("leaf", C.c_int32), ("max_def", C.c_int32), ("max_rep", C.c_int32), ("reserved", C.c_int32)]


class ChunkMeta(C.Structure):
    _fields_ = [
        ("start", C.c_int64),
        ("total_compressed_size", C.c_int64),
        ("total_uncompressed_size", C.c_int64),
        ("data_page_offset", C.c_int64),
        ("num_values", C.c_int64),
        ("has_dict_page_offset", C.c_int32),
        ("codec", C.c_int32),
        ("type", C.c_int32),
        ("reserved", C.c_int32),
    ]


class AssembleArgs(C.Structure):
    """pqg_assemble_args (include/pqgpu.h, K8)."""
    _fields_ = [("def_levels", C.c_void_p), ("rep_levels", C.c_void_p), ("values", C.c_void_p),
                ("num_slots", C.c_int64), ("max_def", C.c_int32), ("boundary_level", C.c_int32),
                ("value_width", C.c_int32), ("reserved", C.c_int32),
                ("validity", C.c_void_p), ("values_spaced", C.c_void_p), ("offsets", C.c_void_p),
                ("num_valid", C.c_int64), ("null_count", C.c_int64), ("num_boundaries", C.c_int64)]


class ListArgs(C.Structure):
    """pqg_list_args (include/pqgpu.h, K8 list export)."""
    _fields_ = [("def_levels", C.c_void_p), ("rep_levels", C.c_void_p), ("values", C.c_void_p),
                ("num_slots", C.c_int64), ("max_def", C.c_int32), ("list_def", C.c_int32),
                ("elem_def", C.c_int32), ("value_width", C.c_int32),
                ("list_validity", C.c_void_p), ("list_offsets", C.c_void_p), ("elem_validity", C.c_void_p),
                ("elem_values", C.c_void_p),
                ("num_rows", C.c_int64), ("num_elements", C.c_int64), ("num_valid", C.c_int64),
                ("null_lists", C.c_int64)]


def status_name(code):
    return STATUS.get(int(code), str(code))
