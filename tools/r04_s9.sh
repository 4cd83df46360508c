#!/bin/bash
# Round-4 session 9: block_walk over LDS chunks, k_str_copy through LDS; snappy batches of up to 3 windows, far sources loaded
# ahead of the doubling: snappy parity, C3 / C4 / C5 bench lines, C4 phase counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_snappy.py tests/test_snappy_split.py tests/test_gpu_parity.py tests/test_delta_strings.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r04_s9_tests.txt 2>&1 || { tail -40 gpurun_out/r04_s9_tests.txt; exit 1; }
tail -2 gpurun_out/r04_s9_tests.txt
run() {  # name, config
  timeout -k 10 300 python3 -u bench.py --only $2 --steps 5 --warmup 2 --no-cpu \
    > gpurun_out/r04_s9_$1.json 2> gpurun_out/r04_s9_$1.err || { tail -5 gpurun_out/r04_s9_$1.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r04_s9_$1.json')); r=d['roofline']
print('$1', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.03})"
}
run c4 c4
run c3 c3
run c5 c5
PQG_LIB=$PWD/parquet-go_amd/csrc/libpqgpu_prof.so timeout -k 10 300 python3 -u tools/phase_probe.py 10000000 c4 \
  > gpurun_out/r04_s9_phase_c4.txt 2>&1 || { tail -5 gpurun_out/r04_s9_phase_c4.txt; exit 1; }
tail -3 gpurun_out/r04_s9_phase_c4.txt
