#!/bin/bash
# Round-4 session 13: block-walk phase timers (C4), unconditional staging loads
# in k_dict4 / DBP / levels / k_snap_seg; C2 / C3 / C4 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/parquet-go_amd/csrc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r04_s13_tests.txt 2>&1 || { tail -40 gpurun_out/r04_s13_tests.txt; exit 1; }
tail -1 gpurun_out/r04_s13_tests.txt
PQG_LIB=$L/libpqgpu_prof.so timeout -k 10 300 python3 -u tools/phase_probe.py 10000000 c4 \
  > gpurun_out/r04_s13_phase_c4.txt 2>&1 || { tail -5 gpurun_out/r04_s13_phase_c4.txt; exit 1; }
tail -1 gpurun_out/r04_s13_phase_c4.txt
run() {  # name, config
  timeout -k 10 300 python3 -u bench.py --only $2 --steps 5 --warmup 2 --no-cpu \
    > gpurun_out/r04_s13_$1.json 2> gpurun_out/r04_s13_$1.err || { tail -5 gpurun_out/r04_s13_$1.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r04_s13_$1.json')); r=d['roofline']
print('$1', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.03})"
}
run c2 c2
run c3 c3
run c4 c4
echo done
