#!/bin/bash
# Round-3 session 16: snappy chain by pointer doubling + dense threshold 8 (default), 8 KiB ring variant;
# parity of the snappy, levels and string paths.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/parquet-go_amd/csrc
timeout -k 10 700 python3 -u -m pytest tests/test_snappy.py tests/test_snappy_split.py tests/test_levels.py tests/test_gpu_parity.py tests/test_delta_strings.py tests/test_assemble.py tests/test_boundary.py -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/r03_s16_tests.txt 2>&1 || { tail -30 gpurun_out/r03_s16_tests.txt; exit 1; }
tail -2 gpurun_out/r03_s16_tests.txt
for v in d8 default r8; do
  lib=$L/libpqgpu_$v.so; [ $v = default ] && lib=$L/libpqgpu.so
  for c in c3 c4 c2; do
    A="--only $c"; [ $c = c2 ] && A="--configs="
    PQG_LIB=$lib timeout -k 10 300 python3 -u bench.py $A --steps 5 --warmup 2 --no-cpu \
      > gpurun_out/r03_s16_${v}_$c.json 2> gpurun_out/r03_s16_${v}_$c.err || { tail -5 gpurun_out/r03_s16_${v}_$c.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/r03_s16_${v}_$c.json')); r=d['roofline']
print('$v $c', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.05})"
    [ $c = c4 ] && [ $v = r8 ] && break
  done
done
