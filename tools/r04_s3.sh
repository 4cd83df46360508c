#!/bin/bash
# Round-4 session 3: k_dict4 phase counters (-DPQG_PROFILE build) on C2 b=8,
# b=12 and b=20 alone (100M rows each), and the levels stage's.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for b in 8 12 20; do
  PQG_LIB=$PWD/parquet-go_amd/csrc/libpqgpu_prof.so timeout -k 10 200 python3 -u tools/phase_probe.py 100000000 c2:$b \
    > gpurun_out/r04_s3_b$b.txt 2>&1 || { tail -5 gpurun_out/r04_s3_b$b.txt; exit 1; }
  tail -2 gpurun_out/r04_s3_b$b.txt
done
