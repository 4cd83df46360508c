"""Writes tests/golden/unsigned.parquet: a small pyarrow-written file whose INT32 /
INT64 columns carry the unsigned logical types (INTEGER(isSigned=false) +
ConvertedType UINT_8/UINT_32/UINT_64) that make parquet-go box values as uint32 /
uint64 (getInt32ValuesDecoder / getInt64ValuesDecoder, chunk_reader.go:99-141).
Run here (pyarrow is a container-only tool); the file is committed."""
import io
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

t = pa.table({"u32": pa.array(np.array([1, 2**32 - 1, 7, 2**31], np.uint32)),
              "u64": pa.array(np.array([2**64 - 1, 0, 5, 2**63], np.uint64)),
              "i32": pa.array(np.array([-1, 2, 3, -(2**31)], np.int32)),
              "u8": pa.array(np.array([255, 0, 1, 128], np.uint8)),
              "i64": pa.array(np.array([-1, 0, 2**62, -(2**63)], np.int64))})
b = io.BytesIO()
pq.write_table(t, b, use_dictionary=["u32"], compression="none")
open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "unsigned.parquet"), "wb").write(b.getvalue())
