#!/bin/bash
# Round-4 session 18: the tag-by-tag literal path without the history
# read-back (GPU snappy tests), then dense-threshold A/B on C3 / C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_snappy.py tests/test_snappy_split.py tests/test_gpu_parity.py > gpurun_out/s18_tests.log 2>&1 \
  || { tail -20 gpurun_out/s18_tests.log; exit 1; }
tail -2 gpurun_out/s18_tests.log
PQG_LIB=$PWD/parquet-go_amd/csrc/libpqgpu_prof.so timeout -k 10 300 python3 -u tools/phase_probe.py 100000000 c3 \
  > gpurun_out/s18_phase_c3.txt 2>&1 || { tail -5 gpurun_out/s18_phase_c3.txt; exit 1; }
cat gpurun_out/s18_phase_c3.txt
for CFG in c3 c4; do
  for VAR in d2 d4; do VAR=$VAR CFG=$CFG bash tools/r04_ab.sh || exit 1; done
done
