#!/bin/bash
# Round-3 session 22: DPP prefix max in the multi-run expander (pqg_hybrid.h).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/r03_s22_tests.txt 2>&1 || { tail -30 gpurun_out/r03_s22_tests.txt; exit 1; }
tail -2 gpurun_out/r03_s22_tests.txt
for c in c5 c4; do
  timeout -k 10 300 python3 -u bench.py --only $c --steps 5 --warmup 2 --no-cpu \
    > gpurun_out/r03_s22_$c.json 2> gpurun_out/r03_s22_$c.err || { tail -5 gpurun_out/r03_s22_$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r03_s22_$c.json')); r=d['roofline']
print('$c', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.03})"
done
