#!/bin/bash
# Round-4 session 2: big-page parts (k_part_plan, k_level_long, k_walk_long):
# the big-page parity tests first, then every GPU test, then short benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_big_pages.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r04_s2_big.txt 2>&1 || { tail -40 gpurun_out/r04_s2_big.txt; exit 1; }
tail -3 gpurun_out/r04_s2_big.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r04_s2_tests.txt 2>&1 || { tail -30 gpurun_out/r04_s2_tests.txt; exit 1; }
tail -2 gpurun_out/r04_s2_tests.txt
for c in c1_1page c1 c2 c5; do
  timeout -k 10 300 python3 -u bench.py --only $c --steps 5 --warmup 2 --no-cpu \
    > gpurun_out/r04_s2_$c.json 2> gpurun_out/r04_s2_$c.err || { tail -5 gpurun_out/r04_s2_$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r04_s2_$c.json')); r=d['roofline']
print('$c', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.03})"
done
