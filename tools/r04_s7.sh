#!/bin/bash
# Round-4 session 7: GPU inflate (k_inflate) parity, the whole -m gpu suite,
# C2 / C2 run-heavy with the wave level decoder back as the only one, part
# planning folded into k_nn_scan.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gzip.py tests/test_boundary.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r04_s7_gzip.txt 2>&1 || { tail -40 gpurun_out/r04_s7_gzip.txt; exit 1; }
tail -2 gpurun_out/r04_s7_gzip.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r04_s7_tests.txt 2>&1 || { tail -40 gpurun_out/r04_s7_tests.txt; exit 1; }
tail -2 gpurun_out/r04_s7_tests.txt
run() {  # name, config
  timeout -k 10 300 python3 -u bench.py --only $2 --steps 5 --warmup 2 --no-cpu \
    > gpurun_out/r04_s7_$1.json 2> gpurun_out/r04_s7_$1.err || { tail -5 gpurun_out/r04_s7_$1.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r04_s7_$1.json')); r=d['roofline']
print('$1', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.03})"
}
run c2 c2
run c2rh c2_run_heavy
