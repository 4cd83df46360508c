#!/bin/bash
# Round-4 session 1: the GPU tests on this round's first build, then short
# bench runs of C2, the C1 one-page variant and C2 run-heavy (no CPU leg).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r04_s1_tests.txt 2>&1 || { tail -30 gpurun_out/r04_s1_tests.txt; exit 1; }
tail -2 gpurun_out/r04_s1_tests.txt
for c in c2 c1 c1_1page c2_run_heavy; do
  timeout -k 10 300 python3 -u bench.py --only $c --steps 5 --warmup 2 --no-cpu \
    > gpurun_out/r04_s1_$c.json 2> gpurun_out/r04_s1_$c.err || { tail -5 gpurun_out/r04_s1_$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r04_s1_$c.json')); r=d['roofline']
print('$c', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.03})"
done
