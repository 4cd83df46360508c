#!/bin/bash
# Round-3 session 6: k_dict4 experiment switches (no store / no gather / no decode) at C2 b = 8 and 16.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/parquet-go_amd/csrc
for b in 8 16; do for v in default ns ng nd; do
  lib=$L/libpqgpu_$v.so; [ $v = default ] && lib=$L/libpqgpu.so
  PQG_LIB=$lib timeout -k 10 200 python3 -u bench.py --configs= --bits $b --steps 10 --warmup 2 --no-cpu --no-verify \
    > gpurun_out/r03_s6_b${b}_$v.json 2> gpurun_out/r03_s6_b${b}_$v.err || { tail -5 gpurun_out/r03_s6_b${b}_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r03_s6_b${b}_$v.json')); r=d['roofline']
print('b=$b $v', d['value'], 'GB/s', d['ms_per_step'], 'ms values', r['stage_ms']['values'])"
done; done
exit 0
