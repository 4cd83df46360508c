#!/bin/bash
# Round-3 session 1: GPU tests, C3/C4 snappy after the sc1 change, C4 phase counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
{ command -v go; go version; } > gpurun_out/go_probe.txt 2>&1 || true
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r03_pytest_gpu_s1.log 2>&1 || exit $?
for cfg in c4 c3; do
  timeout -k 10 300 python3 -u bench.py --only $cfg --steps 5 --warmup 2 --no-cpu \
    > gpurun_out/r03_s1_$cfg.json 2> gpurun_out/r03_s1_$cfg.err || exit $?
done
PQG_LIB=$PWD/parquet-go_amd/csrc/libpqgpu_prof.so timeout -k 10 300 python3 -u tools/phase_probe.py 3000000 c4 \
  > gpurun_out/r03_s1_phase_c4.txt 2>&1 || exit $?
exit 0
