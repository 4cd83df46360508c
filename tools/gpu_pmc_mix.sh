#!/bin/bash
# Instruction-mix PMC passes (two separate rocprofv3 runs) over one C2 width.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ARGS=${MIX_ARGS:---bits 8 --configs= --steps 2 --warmup 1 --no-cpu --no-verify}
PMC="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  PMC_NAME=mixA PMC_ARGS="$ARGS" bash tools/gpu_pmc.sh || exit $?
PMC="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_WAVE_CYCLES" \
  PMC_NAME=mixB PMC_ARGS="$ARGS" bash tools/gpu_pmc.sh || exit $?
exit 0
