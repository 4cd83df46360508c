#!/bin/bash
# Round-4 session 16: non-temporal stores for every decoded output; k_str_copy
# stages PLAIN / DLBA sources in LDS.  Whole -m gpu suite, every config.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r04_s16_tests.txt 2>&1 || { tail -40 gpurun_out/r04_s16_tests.txt; exit 1; }
tail -1 gpurun_out/r04_s16_tests.txt
run() {  # name, config
  timeout -k 10 300 python3 -u bench.py --only $2 --steps 5 --warmup 2 --no-cpu \
    > gpurun_out/r04_s16_$1.json 2> gpurun_out/r04_s16_$1.err || { tail -5 gpurun_out/r04_s16_$1.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r04_s16_$1.json')); r=d['roofline']
print('$1', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.03})"
}
run c2 c2
run c3 c3
run c4 c4
run c5 c5
run c1 c1
run c1_1page c1_1page
run c2rh c2_run_heavy
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_s16_prof_c4 -o c4 -- python3 -u bench.py --only c4 --steps 5 --warmup 2 --no-cpu \
  > gpurun_out/r04_s16_prof_c4.log 2>&1 || { tail -5 gpurun_out/r04_s16_prof_c4.log; exit 1; }
echo done
