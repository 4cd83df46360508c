#!/bin/bash
# Round-3 session 14: snappy phase counters on C3 / C4 (profile build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in c3 c4; do
  PQG_LIB=$PWD/parquet-go_amd/csrc/libpqgpu_prof.so timeout -k 10 300 python3 -u tools/phase_probe.py 20000000 $c > gpurun_out/r03_s14_$c.txt 2>&1 || { tail -5 gpurun_out/r03_s14_$c.txt; exit 1; }
  tail -3 gpurun_out/r03_s14_$c.txt
done
