#!/bin/bash
# rocprofv3 kernel-trace summaries, one run per config (bench.py --only <cfg>).
# Output: gpurun_out/prof_<cfg>/ (+ gpurun_out/prof_<cfg>.json, the bench line).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in ${CONFIGS:-c2 c1 c3 c4 c5}; do
  timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$cfg -o run -- \
      python3 -u bench.py --only $cfg --steps ${STEPS:-5} --warmup 2 --no-cpu --no-verify $EXTRA \
      > gpurun_out/prof_$cfg.json 2> gpurun_out/prof_$cfg.err
  rc=$?
  echo "$cfg rocprof rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
exit 0
