#!/bin/bash
# Round-4 session 23: DBP two-dword value reads for widths <= 32 —
# GPU snappy/DBP tests, C3/C4/C5 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_snappy.py tests/test_snappy_split.py tests/test_gpu_parity.py > gpurun_out/s23_tests.log 2>&1 \
  || { tail -30 gpurun_out/s23_tests.log; exit 1; }
tail -2 gpurun_out/s23_tests.log
for CFG in c3 c5; do
  timeout -k 10 400 python3 -u bench.py --only $CFG --steps 5 --warmup 2 --no-cpu > gpurun_out/s23_$CFG.json 2> gpurun_out/s23_$CFG.err \
    || { tail -5 gpurun_out/s23_$CFG.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/s23_$CFG.json')); r=d['roofline']
print('$CFG', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.02})"
done
