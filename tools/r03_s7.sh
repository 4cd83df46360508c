#!/bin/bash
# Round-3 session 7: k_dict4 pair-loop phase split at b = 8; instruction-mix PMC pass at b = 8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/parquet-go_amd/csrc
PQG_LIB=$L/libpqgpu_prof.so timeout -k 10 200 python3 -u tools/phase_probe.py 100000000 c2:8 > gpurun_out/r03_s7_phase_b8.txt 2>&1 || exit $?
tail -1 gpurun_out/r03_s7_phase_b8.txt
ARGS="--bits 8 --configs= --steps 2 --warmup 1 --no-cpu --no-verify"
PMC="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
  PMC_NAME=r03_mixA PMC_ARGS="$ARGS" bash tools/gpu_pmc.sh || exit $?
PMC="SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
  PMC_NAME=r03_mixB PMC_ARGS="$ARGS" bash tools/gpu_pmc.sh || exit $?
PMC="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES" PMC_NAME=r03_lds PMC_ARGS="$ARGS" bash tools/gpu_pmc.sh || exit $?
exit 0
