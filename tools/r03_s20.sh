#!/bin/bash
# Round-3 session 20: k_page_chain / k_page_list with one block scan per job.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/r03_s20_tests.txt 2>&1 || { tail -30 gpurun_out/r03_s20_tests.txt; exit 1; }
tail -2 gpurun_out/r03_s20_tests.txt
for c in c2 c3 c4 c5; do
  A="--only $c"; [ $c = c2 ] && A="--configs="
  timeout -k 10 300 python3 -u bench.py $A --steps 10 --warmup 2 --no-cpu \
    > gpurun_out/r03_s20_$c.json 2> gpurun_out/r03_s20_$c.err || { tail -5 gpurun_out/r03_s20_$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r03_s20_$c.json')); r=d['roofline']
print('$c', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.02})"
done
