#!/bin/bash
# Round-4 session 6: wave-synchronous window refills (lane levels, walker),
# walker's unconditional ring loads, k_dict4 without its LDS output buffer.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_levels.py tests/test_big_pages.py tests/test_gpu_parity.py tests/test_assemble.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r04_s6_tests.txt 2>&1 || { tail -40 gpurun_out/r04_s6_tests.txt; exit 1; }
tail -2 gpurun_out/r04_s6_tests.txt
run() {  # name, env, config
  env $2 timeout -k 10 300 python3 -u bench.py --only $3 --steps 5 --warmup 2 --no-cpu \
    > gpurun_out/r04_s6_$1.json 2> gpurun_out/r04_s6_$1.err || { tail -5 gpurun_out/r04_s6_$1.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r04_s6_$1.json')); r=d['roofline']
print('$1', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.03})"
}
run c2_lane PQG_LEVELS=lane c2
run c2_wave PQG_LEVELS=wave c2
run c2rh_lane PQG_LEVELS=lane c2_run_heavy
run c5_lane PQG_LEVELS=lane c5
