#!/bin/bash
# A/B of a variant library against the default on one config (bench lines
# only): VAR=<variant name> CFG=<config>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/parquet-go_amd/csrc
for rep in a b; do
  for lib in libpqgpu libpqgpu_$VAR; do
    PQG_LIB=$L/$lib.so timeout -k 10 300 python3 -u bench.py --only $CFG --steps 5 --warmup 2 --no-cpu \
      > gpurun_out/ab_${lib}_$rep.json 2> gpurun_out/ab_${lib}_$rep.err || { tail -5 gpurun_out/ab_${lib}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/ab_${lib}_$rep.json')); r=d['roofline']
print('$lib $rep', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.02})"
  done
done
