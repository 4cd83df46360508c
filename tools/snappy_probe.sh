#!/bin/bash
# C3 / C4 / C5 with the default build and experiment builds of the snappy stage.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in default $VARIANTS; do
  lib=parquet-go_amd/csrc/libpqgpu_$v.so; [ "$v" = default ] && lib=parquet-go_amd/csrc/libpqgpu.so
  for cfg in c3 c4 c5; do
    PQG_LIB=$PWD/$lib timeout -k 10 300 python3 -u bench.py --only $cfg --steps 5 --warmup 2 --no-cpu > gpurun_out/snp_${cfg}_$v.json 2> gpurun_out/snp_${cfg}_$v.err || exit $?
  done
done
