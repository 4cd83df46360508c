#!/bin/bash
# One GPU session: GPU tests, then a bench run, each under its own time limit.
# Stops at the first GPU fault / abort / timeout (exit 124, 134, 137, 139).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
TESTS=${TESTS:-tests}
timeout -k 10 ${TEST_TIMEOUT:-420} python -u -m pytest $TESTS -m gpu -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if fatal $rc; then echo "stopping after fatal pytest exit"; exit $rc; fi
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-420} python -u bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?
  echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
  if fatal $rc; then exit $rc; fi
fi
exit 0
