#!/bin/bash
# Round-4 session 15: C2 variants -- non-temporal k_dict4 output stores
# (PQG_DICT_NT: keep the b = 20 dictionary in L2), the level decoder at 4
# waves/SIMD without spills (PQG_LEVELS_WPE=4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/parquet-go_amd/csrc
PQG_LIB=$L/libpqgpu_nt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "c2 or dict" --timeout 120 --timeout-method thread \
  > gpurun_out/r04_s15_tests_nt.txt 2>&1 || { tail -20 gpurun_out/r04_s15_tests_nt.txt; exit 1; }
tail -1 gpurun_out/r04_s15_tests_nt.txt
PQG_LIB=$L/libpqgpu_lw4.so timeout -k 10 300 python -u -m pytest tests/test_levels.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r04_s15_tests_lw4.txt 2>&1 || { tail -20 gpurun_out/r04_s15_tests_lw4.txt; exit 1; }
tail -1 gpurun_out/r04_s15_tests_lw4.txt
run() {  # name, config, library
  PQG_LIB=$3 timeout -k 10 300 python3 -u bench.py --only $2 --steps 5 --warmup 2 --no-cpu \
    > gpurun_out/r04_s15_$1.json 2> gpurun_out/r04_s15_$1.err || { tail -5 gpurun_out/r04_s15_$1.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r04_s15_$1.json')); r=d['roofline']
print('$1', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.03})"
}
run c2 c2 $L/libpqgpu.so
run c2_nt c2 $L/libpqgpu_nt.so
run c2_lw4 c2 $L/libpqgpu_lw4.so
run c2b c2 $L/libpqgpu.so
run c2_nt_b c2 $L/libpqgpu_nt.so
echo done
