#!/bin/bash
# Round-3 session 3: GPU tests with k_dict4, C2 A/B (k_values<1> vs k_dict4), C4 kernel summary + snappy phases.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r03_s3_pytest.log 2>&1 || { tail -30 gpurun_out/r03_s3_pytest.log; exit 1; }
tail -2 gpurun_out/r03_s3_pytest.log
for d in 0 1; do
  PQG_DICT4=$d timeout -k 10 300 python3 -u bench.py --configs= --steps 10 --warmup 2 --no-cpu \
    > gpurun_out/r03_s3_c2_dict$d.json 2> gpurun_out/r03_s3_c2_dict$d.err || { tail -5 gpurun_out/r03_s3_c2_dict$d.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r03_s3_c2_dict$d.json')); r=d['roofline']
print('dict4=$d', d['value'], 'GB/s', d['ms_per_step'], 'ms', {k: v for k, v in r['stage_ms'].items() if v > 0.02})"
done
CONFIGS="c4" STEPS=3 bash tools/prof_all.sh || exit $?
PQG_LIB=$PWD/parquet-go_amd/csrc/libpqgpu_prof.so timeout -k 10 300 python3 -u tools/phase_probe.py 50000000 c4 \
  > gpurun_out/r03_s3_phase_c4.txt 2>&1 || exit $?
exit 0
