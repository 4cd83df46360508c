#!/bin/bash
# Round-4 session 19: speculative DBP header walk — the GPU suite, C3 bench,
# C3 phase counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
  > gpurun_out/s19_tests.log 2>&1 || { tail -30 gpurun_out/s19_tests.log; exit 1; }
tail -2 gpurun_out/s19_tests.log
for rep in a b; do
  timeout -k 10 300 python3 -u bench.py --only c3 --steps 10 --warmup 2 --no-cpu > gpurun_out/s19_c3_$rep.json 2> gpurun_out/s19_c3_$rep.err \
    || { tail -5 gpurun_out/s19_c3_$rep.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/s19_c3_$rep.json')); r=d['roofline']
print('c3 $rep', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.02})"
done
PQG_LIB=$PWD/parquet-go_amd/csrc/libpqgpu_prof.so timeout -k 10 300 python3 -u tools/phase_probe.py 100000000 c3 \
  > gpurun_out/s19_phase_c3.txt 2>&1 || { tail -5 gpurun_out/s19_phase_c3.txt; exit 1; }
cat gpurun_out/s19_phase_c3.txt
