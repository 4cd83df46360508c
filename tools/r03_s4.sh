#!/bin/bash
# Round-3 session 4: k_dict4 vs k_values<1> per C2 width, k_dict4 phase counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in 8 16; do for d in 0 1; do
  PQG_DICT4=$d timeout -k 10 200 python3 -u bench.py --configs= --bits $b --steps 10 --warmup 2 --no-cpu --no-verify \
    > gpurun_out/r03_s4_b${b}_dict$d.json 2> gpurun_out/r03_s4_b${b}_dict$d.err || { tail -5 gpurun_out/r03_s4_b${b}_dict$d.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r03_s4_b${b}_dict$d.json')); r=d['roofline']
print('b=$b dict4=$d', d['value'], 'GB/s', d['ms_per_step'], 'ms', {k: v for k, v in r['stage_ms'].items() if v > 0.02})"
done; done
for b in 8 16; do
PQG_LIB=$PWD/parquet-go_amd/csrc/libpqgpu_prof.so timeout -k 10 200 python3 -u tools/phase_probe.py 100000000 c2:$b \
  > gpurun_out/r03_s4_phase_b$b.txt 2>&1 || exit $?
done
exit 0
