#!/bin/bash
# Round-4 session 8: the whole -m gpu suite (DBA padding-lane fix), C2 / C2
# run-heavy / C3 / C4 bench lines, and the snappy phase counters on C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r04_s8_tests.txt 2>&1 || { tail -40 gpurun_out/r04_s8_tests.txt; exit 1; }
tail -2 gpurun_out/r04_s8_tests.txt
run() {  # name, config
  timeout -k 10 300 python3 -u bench.py --only $2 --steps 5 --warmup 2 --no-cpu \
    > gpurun_out/r04_s8_$1.json 2> gpurun_out/r04_s8_$1.err || { tail -5 gpurun_out/r04_s8_$1.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r04_s8_$1.json')); r=d['roofline']
print('$1', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.03})"
}
run c2 c2
run c2rh c2_run_heavy
run c3 c3
run c4 c4
PQG_LIB=$PWD/parquet-go_amd/csrc/libpqgpu_prof.so timeout -k 10 300 python3 -u tools/phase_probe.py 10000000 c4 \
  > gpurun_out/r04_s8_phase_c4.txt 2>&1 || { tail -5 gpurun_out/r04_s8_phase_c4.txt; exit 1; }
tail -3 gpurun_out/r04_s8_phase_c4.txt
