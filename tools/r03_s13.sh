#!/bin/bash
# Round-3 session 13: DBP header walk from one uniform stage read; level chains by pointer doubling.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/parquet-go_amd/csrc
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_boundary.py tests/test_levels.py -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/r03_s13_tests.txt 2>&1 || { tail -30 gpurun_out/r03_s13_tests.txt; exit 1; }
tail -3 gpurun_out/r03_s13_tests.txt
for v in serial new; do
  lib=$L/libpqgpu_$v.so; [ $v = new ] && lib=$L/libpqgpu.so
  for c in c2 c3; do
    if [ $c = c2 ]; then A="--configs="; else A="--only c3"; fi
    PQG_LIB=$lib timeout -k 10 300 python3 -u bench.py $A --steps 10 --warmup 2 --no-cpu \
      > gpurun_out/r03_s13_${v}_$c.json 2> gpurun_out/r03_s13_${v}_$c.err || { tail -5 gpurun_out/r03_s13_${v}_$c.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/r03_s13_${v}_$c.json')); r=d['roofline']
print('$v $c', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.02})"
  done
done
MIX_ARGS="--only c3 --c3-rows 200000000 --steps 2 --warmup 1 --no-cpu --no-verify" bash tools/gpu_pmc_mix.sh
mkdir -p gpurun_out/pmc_c3 && mv gpurun_out/pmc/* gpurun_out/pmc_c3/
MIX_ARGS="--bits 8 --configs= --steps 2 --warmup 1 --no-cpu --no-verify" bash tools/gpu_pmc_mix.sh
