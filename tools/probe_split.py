import sys; sys.path[:0]=[".", "parquet-go_amd", "tests"]
import pqgpu
from gen import pqwrite as W
dec=pqgpu.GpuDecoder(0)
data=W.config_c4(rows=60000, vocab=20000, rows_per_page=60000, seed=7, dict_limit=1<<20)[0]
pf=pqgpu.ParquetFile(data); dev=dec.upload(pf.data)
r=dec.decode_jobs([pqgpu.device_job(pf,0,0,dev)])
for p in dec.pages(0): print(p.page_type, p.compressed_size, p.uncompressed_size, hex(p.flags))
