#!/bin/bash
# Round-4 session 17: dictionary pages back on the global-window walk;
# unconditional loads in k_page_cands / k_cand_parse / long literals / the LDS
# dictionary stage.  Tests; C2..C5 lines; C3 / C5 with the guarded long-literal
# loads (libpqgpu_ll0) for A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/parquet-go_amd/csrc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r04_s17_tests.txt 2>&1 || { tail -40 gpurun_out/r04_s17_tests.txt; exit 1; }
tail -1 gpurun_out/r04_s17_tests.txt
run() {  # name, config, library
  PQG_LIB=$3 timeout -k 10 300 python3 -u bench.py --only $2 --steps 5 --warmup 2 --no-cpu \
    > gpurun_out/r04_s17_$1.json 2> gpurun_out/r04_s17_$1.err || { tail -5 gpurun_out/r04_s17_$1.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r04_s17_$1.json')); r=d['roofline']
print('$1', d['value'], 'GB/s', d['ms_per_step'], 'ms', d.get('verified_bit_exact'), {k: v for k, v in r['stage_ms'].items() if v > 0.03})"
}
run c2 c2 $L/libpqgpu.so
run c3 c3 $L/libpqgpu.so
run c3_ll0 c3 $L/libpqgpu_ll0.so
run c4 c4 $L/libpqgpu.so
run c5 c5 $L/libpqgpu.so
run c5_ll0 c5 $L/libpqgpu_ll0.so
echo done
