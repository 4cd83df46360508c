#!/bin/bash
# One rocprofv3 PMC pass (counters in $PMC) over a short bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL ${PMC_TIMEOUT:-120} rocprofv3 --pmc $PMC --output-format csv -d gpurun_out/pmc -o ${PMC_NAME:-pass} -- \
    python3 -u bench.py ${PMC_ARGS:---rows 20000000 --steps 2 --warmup 1 --no-cpu --no-verify} > gpurun_out/pmc_${PMC_NAME:-pass}.json 2> gpurun_out/pmc_${PMC_NAME:-pass}.err
rc=$?
echo "pmc rc=$rc"
exit $rc
