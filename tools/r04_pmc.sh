#!/bin/bash
# Round-4 PMC traffic: FETCH_SIZE and WRITE_SIZE passes (separate rocprofv3
# runs, one counter set each) over the default-size workload of every config,
# then LDS bank-conflict passes; the FETCH_SIZE calibration of 4-byte loads and
# gathers (tools/fetch_calib.hip).  Output: gpurun_out/pmc/<name>_*.csv and
# gpurun_out/pmc_<name>.json (the bench line of the pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in ${PMC_CONFIGS:-c2 c1 c3 c4 c5}; do
  A="--only $cfg --steps 2 --warmup 1 --no-cpu --no-verify"
  PMC=FETCH_SIZE PMC_NAME=fetch_$cfg PMC_ARGS="$A" PMC_TIMEOUT=300 bash tools/gpu_pmc.sh || exit $?
  PMC=WRITE_SIZE PMC_NAME=write_$cfg PMC_ARGS="$A" PMC_TIMEOUT=300 bash tools/gpu_pmc.sh || exit $?
done
for cfg in ${LDS_CONFIGS:-c2 c3 c4}; do
  PMC="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES" PMC_NAME=lds_$cfg \
    PMC_ARGS="--only $cfg --steps 2 --warmup 1 --no-cpu --no-verify" PMC_TIMEOUT=300 bash tools/gpu_pmc.sh || exit $?
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o calib -- ./tools/fetch_calib \
  > gpurun_out/pmc_calib.log 2>&1 || exit $?
exit 0
