#!/bin/bash
# round-6 final: rocprofv3 kernel summaries, one config per run on one stream
# (CFGS: the configs of this call)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ONLY_ARGS="--streams 1" TAG=r06_prof bash tools/gpu_steps.sh $(for c in ${CFGS:-c2 c2_run_heavy c1 c1_1page c3 c3_gzip c4 c5}; do echo prof:$c; done)
