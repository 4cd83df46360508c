#!/bin/bash
# One GPU iteration: TESTS (pytest args, "" = skip), then bench.py --only for each
# config in CONFIGS, outputs tagged TAG under gpurun_out/.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-iter}
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -2 gpurun_out/${TAG}_pytest.log
fi
for cfg in $CONFIGS; do
  timeout -k 10 ${BENCH_TIMEOUT:-300} python3 -u bench.py --only $cfg --steps ${STEPS:-5} --warmup 2 --no-cpu $BENCH_ARGS \
    > gpurun_out/${TAG}_$cfg.json 2> gpurun_out/${TAG}_$cfg.err || { tail -20 gpurun_out/${TAG}_$cfg.err; exit 2; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_$cfg.json')); r=d['roofline']
print('$cfg', d['value'], 'GB/s', d['ms_per_step'], 'ms', r['kernel'], r['kernel_ms'], {k: v for k, v in r['stage_ms'].items() if v > 0.02})"
done
if [ -n "$EXTRA" ]; then eval "$EXTRA" || exit 3; fi
exit 0
