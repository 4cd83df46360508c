#!/bin/bash
# Round-3 session 2: the span-upload test, C4/C2 kernel summaries, C4 snappy phase counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_boundary.py tests/test_sharding.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r03_s2_pytest.log 2>&1 || { tail -20 gpurun_out/r03_s2_pytest.log; exit 1; }
tail -2 gpurun_out/r03_s2_pytest.log
CONFIGS="c4 c2" STEPS=3 bash tools/prof_all.sh || exit $?
PQG_LIB=$PWD/parquet-go_amd/csrc/libpqgpu_prof.so timeout -k 10 300 python3 -u tools/phase_probe.py 50000000 c4 \
  > gpurun_out/r03_s2_phase_c4.txt 2>&1 || exit $?
exit 0
