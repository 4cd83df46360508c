#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run (one GPU).
# Output: gpurun_out/prof/<run>/..._kernel_stats.csv; copy the summary you want
# judged into profiles/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- \
    python3 -u bench.py ${PROF_ARGS:---steps 5 --warmup 2 --no-cpu --no-verify} > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
rc=$?
echo "rocprof rc=$rc"; cat gpurun_out/prof_bench.json
find gpurun_out/prof -name "*kernel_stats.csv" | head -5
exit $rc
