#!/bin/bash
# Round-3 session 8: k_dict4 with the LDS output buffer: GPU tests, C2 per-width + full, phases, LDS/mix PMC at b = 8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r03_s8_pytest.log 2>&1 || { tail -30 gpurun_out/r03_s8_pytest.log; exit 1; }
tail -2 gpurun_out/r03_s8_pytest.log
L=$PWD/parquet-go_amd/csrc
run() {  # name bench-args env...
  local name=$1 args=$2; shift 2
  env "$@" timeout -k 10 300 python3 -u bench.py --configs= $args --steps 10 --warmup 2 --no-cpu --no-verify \
    > gpurun_out/r03_s8_$name.json 2> gpurun_out/r03_s8_$name.err || { tail -5 gpurun_out/r03_s8_$name.err; return 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r03_s8_$name.json')); r=d['roofline']
print('$name', d['value'], 'GB/s', d['ms_per_step'], 'ms', {k: v for k, v in r['stage_ms'].items() if v > 0.02})"
}
run b8 "--bits 8" || exit 1
run b16 "--bits 16" || exit 1
run b1 "--bits 1" || exit 1
run full "" || exit 1
run full_old "" PQG_DICT4=0 || exit 1
PQG_LIB=$L/libpqgpu_prof.so timeout -k 10 200 python3 -u tools/phase_probe.py 100000000 c2:8 > gpurun_out/r03_s8_phase_b8.txt 2>&1 || exit $?
tail -1 gpurun_out/r03_s8_phase_b8.txt
ARGS="--bits 8 --configs= --steps 2 --warmup 1 --no-cpu --no-verify"
PMC="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
  PMC_NAME=r03_s8_mixA PMC_ARGS="$ARGS" bash tools/gpu_pmc.sh || exit $?
PMC="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES" PMC_NAME=r03_s8_lds PMC_ARGS="$ARGS" bash tools/gpu_pmc.sh || exit $?
exit 0
