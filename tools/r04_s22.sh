#!/bin/bash
# Round-4 session 22: snappy tag-by-tag phase counters on C3 (prof library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PQG_LIB=$PWD/parquet-go_amd/csrc/libpqgpu_prof.so timeout -k 10 300 python3 -u tools/phase_probe.py 100000000 c3 \
  > gpurun_out/s22_phase_c3.txt 2>&1 || { tail -5 gpurun_out/s22_phase_c3.txt; exit 1; }
cat gpurun_out/s22_phase_c3.txt
PQG_LIB=$PWD/parquet-go_amd/csrc/libpqgpu_prof.so timeout -k 10 300 python3 -u tools/phase_probe.py 20000000 c3 \
  > gpurun_out/s22_phase_c3_small.txt 2>&1 || { tail -5 gpurun_out/s22_phase_c3_small.txt; exit 1; }
cat gpurun_out/s22_phase_c3_small.txt
