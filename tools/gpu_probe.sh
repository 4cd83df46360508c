#!/bin/bash
# Measurement session: C2 per-width bench lines, rocprof kernel-trace summaries
# per config, and one LDS bank-conflict PMC pass per config.  Each GPU step has
# its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
if [ -z "$SKIP_WIDTHS" ]; then
  bash tools/c2_widths.sh || exit $?
  echo "widths ok"
fi
if [ -n "$PROF_CONFIGS" ]; then
  CONFIGS="$PROF_CONFIGS" bash tools/prof_all.sh || exit $?
fi
for cfg in $LDS_CONFIGS; do
  PMC="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES" PMC_NAME=lds_$cfg \
    PMC_ARGS="--only $cfg --steps 2 --warmup 1 --no-cpu --no-verify ${LDS_EXTRA}" bash tools/gpu_pmc.sh || exit $?
done
for v in $SNAPPY_VARIANTS; do
  lib=parquet-go_amd/csrc/libpqgpu_$v.so; [ "$v" = default ] && lib=parquet-go_amd/csrc/libpqgpu.so
  for cfg in c3 c4; do
    PQG_LIB=$PWD/$lib timeout -k 10 200 python3 -u bench.py --only $cfg --steps 5 --warmup 2 --no-cpu \
        > gpurun_out/snv_${v}_$cfg.json 2> gpurun_out/snv_${v}_$cfg.err || exit $?
  done
done
exit 0
