#!/bin/bash
# Round-4 measurement: the GPU tests, smoke(), the default bench line,
# rocprofv3 kernel summaries per config (tools/prof_all.sh), then the PMC
# traffic passes (tools/r04_pmc.sh).  Each GPU step has its own limit; stops at
# the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { echo "bench failed"; tail -5 gpurun_out/bench_final.err; exit 1; }
echo bench ok
CONFIGS="${PROF_CONFIGS:-c2 c1 c3 c4 c5}" bash tools/prof_all.sh || exit $?
[ -n "$NO_PMC" ] && exit 0
bash tools/r04_pmc.sh || exit $?
exit 0
