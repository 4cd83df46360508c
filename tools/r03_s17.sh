#!/bin/bash
# Round-3 session 17: level-decoder phase counters on C2 (profile build), b=8 and b=16.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PQG_LIB=$PWD/parquet-go_amd/csrc/libpqgpu_prof.so timeout -k 10 300 python3 -u tools/phase_probe.py 20000000 c2:8 > gpurun_out/r03_s17_c2.txt 2>&1 || { tail -5 gpurun_out/r03_s17_c2.txt; exit 1; }
tail -2 gpurun_out/r03_s17_c2.txt
