#!/bin/bash
# k_snap_wg phase counters (slots 112-127 of pqg_debug_counters) on C4 and C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PQG_LIB=$PWD/parquet-go_amd/csrc/libpqgpu_prof.so
timeout -k 10 200 python3 -u tools/phase_probe.py ${C4_ROWS:-3000000} c4 > gpurun_out/wgp_c4.txt 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/phase_probe.py ${C3_ROWS:-2000000} c3 > gpurun_out/wgp_c3.txt 2>&1 || exit 1
tail -2 gpurun_out/wgp_c4.txt; tail -2 gpurun_out/wgp_c3.txt
