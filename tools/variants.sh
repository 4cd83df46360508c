#!/bin/bash
# bench.py --only <cfg> for each library variant in VARIANTS (default = libpqgpu.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in $VARIANTS; do
  lib=parquet-go_amd/csrc/libpqgpu_$v.so; [ "$v" = default ] && lib=parquet-go_amd/csrc/libpqgpu.so
  for cfg in $CONFIGS; do
    PQG_LIB=$PWD/$lib timeout -k 10 300 python3 -u bench.py --only $cfg --steps 5 --warmup 2 --no-cpu --no-verify \
      > gpurun_out/var_${v}_$cfg.json 2> gpurun_out/var_${v}_$cfg.err || { tail -5 gpurun_out/var_${v}_$cfg.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/var_${v}_$cfg.json')); r=d['roofline']
print('$v $cfg', d['value'], 'GB/s', d['ms_per_step'], 'ms', {k: v for k, v in r['stage_ms'].items() if v > 0.05})"
  done
done
