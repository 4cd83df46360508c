#!/bin/bash
# Round-3 session 21: DPP wave minimum in the snappy segment / link walk.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_snappy.py tests/test_snappy_split.py tests/test_gpu_parity.py tests/test_boundary.py -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/r03_s21_tests.txt 2>&1 || { tail -30 gpurun_out/r03_s21_tests.txt; exit 1; }
tail -2 gpurun_out/r03_s21_tests.txt
for c in c4 c5 c3; do
  timeout -k 10 300 python3 -u bench.py --only $c --steps 5 --warmup 2 --no-cpu \
    > gpurun_out/r03_s21_$c.json 2> gpurun_out/r03_s21_$c.err || { tail -5 gpurun_out/r03_s21_$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r03_s21_$c.json')); r=d['roofline']
print('$c', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.03})"
done
