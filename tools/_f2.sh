#!/bin/bash
# round-6 final: rocprofv3 kernel summaries, one config per run on one stream
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ONLY_ARGS="--streams 1" TAG=r06_prof bash tools/gpu_steps.sh prof:c2 prof:c2_run_heavy prof:c1 prof:c1_1page prof:c3 prof:c3_gzip prof:c4 prof:c5
