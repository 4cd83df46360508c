#!/bin/bash
# Round-3 session 5: GPU tests (k_dict_plan + k_dict4), C2 A/B across dictionary kernels, phases.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r03_s5_pytest.log 2>&1 || { tail -30 gpurun_out/r03_s5_pytest.log; exit 1; }
tail -2 gpurun_out/r03_s5_pytest.log
L=$PWD/parquet-go_amd/csrc
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --configs= --steps 10 --warmup 2 --no-cpu --no-verify \
    > gpurun_out/r03_s5_$name.json 2> gpurun_out/r03_s5_$name.err || { tail -5 gpurun_out/r03_s5_$name.err; return 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r03_s5_$name.json')); r=d['roofline']
print('$name', d['value'], 'GB/s', d['ms_per_step'], 'ms', {k: v for k, v in r['stage_ms'].items() if v > 0.02})"
}
run old PQG_DICT4=0 || exit 1
run d4 PQG_DICT4=1 || exit 1
run w8 PQG_LIB=$L/libpqgpu_w8.so || exit 1
for b in 8 16; do
PQG_LIB=$L/libpqgpu_prof.so timeout -k 10 200 python3 -u tools/phase_probe.py 100000000 c2:$b \
  > gpurun_out/r03_s5_phase_b$b.txt 2>&1 || exit $?
done
exit 0
