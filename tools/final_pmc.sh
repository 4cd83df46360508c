#!/bin/bash
# Round-end PMC passes, one counter set per rocprofv3 run: FETCH_SIZE and
# WRITE_SIZE over the full-size C2 headline (roofline.traffic), then LDS
# bank-conflict passes per config.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
C2ARGS="--configs= --steps 2 --warmup 1 --no-cpu --no-verify"
PMC=FETCH_SIZE PMC_NAME=fetch_c2 PMC_ARGS="$C2ARGS" PMC_TIMEOUT=240 bash tools/gpu_pmc.sh || exit $?
PMC=WRITE_SIZE PMC_NAME=write_c2 PMC_ARGS="$C2ARGS" PMC_TIMEOUT=240 bash tools/gpu_pmc.sh || exit $?
for cfg in ${LDS_CONFIGS:-c2 c3 c4}; do
  PMC="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES" PMC_NAME=lds_$cfg \
    PMC_ARGS="--only $cfg --steps 2 --warmup 1 --no-cpu --no-verify --rows 20000000" PMC_TIMEOUT=240 bash tools/gpu_pmc.sh || exit $?
done
exit 0
