#!/bin/bash
# Experiment builds against the default library: C2 with levels variants, C3 with DBP variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in default $C2_VARIANTS; do
  lib=parquet-go_amd/csrc/libpqgpu_$v.so; [ "$v" = default ] && lib=parquet-go_amd/csrc/libpqgpu.so
  PQG_LIB=$PWD/$lib timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --configs= --no-cpu > gpurun_out/occ_c2_$v.json 2> gpurun_out/occ_c2_$v.err || exit $?
done
for v in default $C3_VARIANTS; do
  lib=parquet-go_amd/csrc/libpqgpu_$v.so; [ "$v" = default ] && lib=parquet-go_amd/csrc/libpqgpu.so
  PQG_LIB=$PWD/$lib timeout -k 10 300 python3 -u bench.py --only c3 --steps 5 --warmup 2 --no-cpu > gpurun_out/occ_c3_$v.json 2> gpurun_out/occ_c3_$v.err || exit $?
done
