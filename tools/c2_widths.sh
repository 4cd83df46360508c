#!/bin/bash
# C2 per-index-width stage times: one bench line per dictionary width b.
# TAG names the output set; PQG_LIB (optional) selects an experiment build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for b in ${WIDTHS:-1 2 4 8 12 16 20}; do
  timeout -k 10 200 python3 -u bench.py --bits $b --steps 10 --warmup 2 --configs= --no-cpu --no-verify \
      > gpurun_out/c2${TAG}_b$b.json 2> gpurun_out/c2${TAG}_b$b.err || exit $?
done
exit 0
