#!/bin/bash
# Round-3 session 12: staged DBP values (C3) parity + bench against the previous build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/parquet-go_amd/csrc
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_boundary.py -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/r03_s12_tests.txt 2>&1 || { tail -30 gpurun_out/r03_s12_tests.txt; exit 1; }
tail -3 gpurun_out/r03_s12_tests.txt
for v in old new; do
  lib=$L/libpqgpu_$v.so; [ $v = new ] && lib=$L/libpqgpu.so
  PQG_LIB=$lib timeout -k 10 300 python3 -u bench.py --only c3 --steps 10 --warmup 2 --no-cpu \
    > gpurun_out/r03_s12_$v.json 2> gpurun_out/r03_s12_$v.err || { tail -5 gpurun_out/r03_s12_$v.err; exit 1; }
  echo $v; tail -c 1500 gpurun_out/r03_s12_$v.json
done
exit 0
