#!/bin/bash
# Round-3 session 15: snappy dense-batch threshold variants on C3 / C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/parquet-go_amd/csrc
for v in default d8 d16 d32; do
  lib=$L/libpqgpu_$v.so; [ $v = default ] && lib=$L/libpqgpu.so
  for c in c3 c4; do
    PQG_LIB=$lib timeout -k 10 300 python3 -u bench.py --only $c --steps 5 --warmup 2 --no-cpu \
      > gpurun_out/r03_s15_${v}_$c.json 2> gpurun_out/r03_s15_${v}_$c.err || { tail -5 gpurun_out/r03_s15_${v}_$c.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/r03_s15_${v}_$c.json')); r=d['roofline']
print('$v $c', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.05})"
  done
done
