#!/bin/bash
# Round-4 session 10: block walk with a 4 KiB read-ahead and most-records
# guesses; k_str_copy through LDS; snappy batch tables aliased into src[].
# C4 / C3 / C5 bench lines with snappy variants (serial v_readlane chain; a
# 4 KiB ring at 3 waves/SIMD; the 8 KiB ring at <= 168 VGPRs), C4 / C3 kernel
# stats and phase counters, FETCH_SIZE calibration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/parquet-go_amd/csrc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_delta_strings.py tests/test_quirks.py tests/test_snappy.py tests/test_snappy_split.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r04_s10_tests.txt 2>&1 || { tail -40 gpurun_out/r04_s10_tests.txt; exit 1; }
tail -2 gpurun_out/r04_s10_tests.txt
PQG_LIB=$L/libpqgpu_r4w3.so timeout -k 10 600 python -u -m pytest tests/test_snappy.py tests/test_snappy_split.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r04_s10_tests_r4w3.txt 2>&1 || { tail -40 gpurun_out/r04_s10_tests_r4w3.txt; exit 1; }
tail -1 gpurun_out/r04_s10_tests_r4w3.txt
run() {  # name, config, library
  PQG_LIB=$3 timeout -k 10 300 python3 -u bench.py --only $2 --steps 5 --warmup 2 --no-cpu \
    > gpurun_out/r04_s10_$1.json 2> gpurun_out/r04_s10_$1.err || { tail -5 gpurun_out/r04_s10_$1.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r04_s10_$1.json')); r=d['roofline']
print('$1', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.03})"
}
run c4 c4 $L/libpqgpu.so
run c4_r4w3 c4 $L/libpqgpu_r4w3.so
run c4_r8w3 c4 $L/libpqgpu_r8w3.so
run c4_sc c4 $L/libpqgpu_sc.so
run c3 c3 $L/libpqgpu.so
run c3_r4w3 c3 $L/libpqgpu_r4w3.so
run c5 c5 $L/libpqgpu.so
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_s10_prof_c4 -o c4 -- python3 -u bench.py --only c4 --steps 5 --warmup 2 --no-cpu \
  > gpurun_out/r04_s10_prof_c4.log 2>&1 || { tail -5 gpurun_out/r04_s10_prof_c4.log; exit 1; }
PQG_LIB=$L/libpqgpu_prof.so timeout -k 10 300 python3 -u tools/phase_probe.py 10000000 c4 \
  > gpurun_out/r04_s10_phase_c4.txt 2>&1 || { tail -5 gpurun_out/r04_s10_phase_c4.txt; exit 1; }
tail -1 gpurun_out/r04_s10_phase_c4.txt
PQG_LIB=$L/libpqgpu_prof.so timeout -k 10 300 python3 -u tools/phase_probe.py 20000000 c3 \
  > gpurun_out/r04_s10_phase_c3.txt 2>&1 || { tail -5 gpurun_out/r04_s10_phase_c3.txt; exit 1; }
tail -1 gpurun_out/r04_s10_phase_c3.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_s10_prof_c3 -o c3 -- python3 -u bench.py --only c3 --steps 5 --warmup 2 --no-cpu \
  > gpurun_out/r04_s10_prof_c3.log 2>&1 || { tail -5 gpurun_out/r04_s10_prof_c3.log; exit 1; }
# FETCH_SIZE calibration for 4-byte loads and gathers (tools/fetch_calib.hip)
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r04_s10_calib -o calib -- ./tools/fetch_calib \
  > gpurun_out/r04_s10_calib.log 2>&1 || { tail -5 gpurun_out/r04_s10_calib.log; exit 1; }
echo done
