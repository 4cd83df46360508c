#!/bin/bash
# Round-3 session 18: page setup split out; walker on a second stream beside the level decode;
# level-decode grid 24 / 20 / 16 waves per CU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_levels.py tests/test_boundary.py tests/test_delta_strings.py tests/test_sharding.py -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/r03_s18_tests.txt 2>&1 || { tail -30 gpurun_out/r03_s18_tests.txt; exit 1; }
tail -2 gpurun_out/r03_s18_tests.txt
for v in 24 20 16; do
  for c in c2 c5; do
    A="--only $c"; [ $c = c2 ] && A="--configs="
    PQG_LEVELS_PER_CU=$v timeout -k 10 300 python3 -u bench.py $A --steps 10 --warmup 2 --no-cpu \
      > gpurun_out/r03_s18_${v}_$c.json 2> gpurun_out/r03_s18_${v}_$c.err || { tail -5 gpurun_out/r03_s18_${v}_$c.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/r03_s18_${v}_$c.json')); r=d['roofline']
print('$v $c', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.02})"
    [ $v != 20 ] && break
  done
done
