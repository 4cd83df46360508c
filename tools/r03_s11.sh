#!/bin/bash
# Round-3 session 11: C2 split over K contexts (streams); k_dict4 3-workgroup variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/parquet-go_amd/csrc
timeout -k 10 400 python3 -u tools/split_probe.py 100000000 1,2,3 > gpurun_out/r03_s11_split.txt 2>&1 || { cat gpurun_out/r03_s11_split.txt; exit 1; }
cat gpurun_out/r03_s11_split.txt
for v in default v3a; do
  lib=$L/libpqgpu_$v.so; [ $v = default ] && lib=$L/libpqgpu.so
  PQG_LIB=$lib timeout -k 10 300 python3 -u bench.py --configs= --steps 10 --warmup 2 --no-cpu --no-verify \
    > gpurun_out/r03_s11_$v.json 2> gpurun_out/r03_s11_$v.err || { tail -5 gpurun_out/r03_s11_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r03_s11_$v.json')); r=d['roofline']
print('$v', d['value'], 'GB/s', d['ms_per_step'], 'ms', {k: v for k, v in r['stage_ms'].items() if v > 0.02})"
done
exit 0
