#!/bin/bash
# One GPU session as a list of steps, each under its own time limit; stops at
# the first failing step (and never starts another GPU step after a fault,
# abort, segfault or time limit).  Output under gpurun_out/$TAG/.
#
#   TAG=r05_s1 bash tools/gpu_steps.sh tests smoke bench probe:c2_run_heavy \
#       prof:c2_run_heavy pmc:c2_run_heavy:FETCH_SIZE pmc:c2_run_heavy:WRITE_SIZE
#
# steps:
#   tests[:<pytest -k expr>]   pytest -m gpu (TESTS= files, default tests/)
#   smoke                      __graft_entry__.smoke()
#   bench[:<name>]             bench.py $BENCH_ARGS  -> bench_<name>.json
#   only:<cfg>[:<name>[:<args>]]  bench.py --only <cfg> $ONLY_ARGS [args, commas for spaces] -> only_<name>.out
#   probe:<cfg>                tools/probe_jobs.py --only <cfg> $PROBE_ARGS
#   prof:<cfg>[:<name>[:<args>]]  rocprofv3 --kernel-trace --stats of bench.py --only <cfg> [args, commas
#                              for spaces] -> prof_<name>.md
#   pmc:<cfg>:<C1,C2,...>      one rocprofv3 --pmc pass of bench.py --only <cfg>
# env: PQG_LIB (library variant), STEPS (bench steps for only/prof/pmc)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-session}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
STEPS_N=${STEPS:-5}
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
run() {  # run <limit> <name> <cmd...>
  local lim=$1 name=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc"
  tail -c 3000 "$OUT/$name.out"
  [ $rc -ne 0 ] && tail -5 "$OUT/$name.err"
  return $rc
}
for step in "$@"; do
  IFS=: read -r kind a1 a2 _rest <<< "$step"
  case $kind in
    tests)
      K=(); [ -n "$a1" ] && K=(-k "$a1")
      run ${TEST_TIMEOUT:-600} pytest python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 120 --timeout-method thread "${K[@]}"
      rc=$?; tail -3 "$OUT/pytest.out" ;;
    smoke) run 300 smoke python -u -c "import __graft_entry__ as g; g.smoke()"; rc=$? ;;
    bench) run ${BENCH_TIMEOUT:-900} "bench_${a1:-main}" python -u bench.py $BENCH_ARGS; rc=$? ;;
    only)  # only:<cfg>[:<name>[:<extra bench args, commas for spaces>]]
      IFS=: read -r _k _c _n ex <<< "$step"
      run 400 "only_${a2:-$a1}" python -u bench.py --only "$a1" --steps "$STEPS_N" --warmup 2 $ONLY_ARGS ${ex//,/ }
      rc=$? ;;
    probe) run 400 "probe_$a1" python -u tools/probe_jobs.py --only "$a1" $PROBE_ARGS; rc=$? ;;
    prof)  # prof:<cfg>[:<name>[:<extra bench args, commas for spaces>]]
      nm=${a2:-$a1}
      IFS=: read -r _k _c _n ex <<< "$step"
      run 400 "prof_$nm" rocprofv3 --kernel-trace --stats -d "$OUT/prof_$nm" -o run -- \
        python3 -u bench.py --only "$a1" --steps "$STEPS_N" --warmup 2 --no-cpu --no-verify $ONLY_ARGS ${ex//,/ }
      rc=$?
      if [ $rc -eq 0 ]; then
        db=$(find "$OUT/prof_$nm" -name "*.db" | head -1)
        csv=$(find "$OUT/prof_$nm" -name "*kernel_stats.csv" | head -1)
        [ -n "$db" ] && python3 tools/prof_summary.py "$db" "$OUT/prof_$nm.md" > /dev/null
        [ -z "$db" ] && [ -n "$csv" ] && cp "$csv" "$OUT/prof_$nm.csv"
      fi ;;
    pmc)
      ctr=${a2//,/ }
      run 300 "pmc_${a1}_${a2//,/_}" rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc" -o "${a1}_${a2//,/_}" -- \
        python3 -u bench.py --only "$a1" --steps 2 --warmup 1 --no-cpu --no-verify $ONLY_ARGS
      rc=$? ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  if [ $rc -ne 0 ]; then
    if fatal $rc; then echo "stopping: fatal exit $rc in $step"; exit $rc; fi
    # failing tests (pytest exit 1) do not stop the measurement steps after them
    if [ "$kind" = tests ] && [ $rc -eq 1 ]; then FAILED=1; continue; fi
    exit $rc
  fi
done
exit ${FAILED:-0}
