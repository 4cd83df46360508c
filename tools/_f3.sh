#!/bin/bash
# round-6 final: FETCH_SIZE / WRITE_SIZE passes (one counter group per run)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ONLY_ARGS="--streams 1" TAG=r06_pmc bash tools/gpu_steps.sh $(for c in ${CFGS:-c2 c2_run_heavy c1 c1_1page c3 c3_gzip c4 c5}; do echo pmc:$c:FETCH_SIZE pmc:$c:WRITE_SIZE; done)
