#!/bin/bash
# round-6 final: the whole GPU suite, smoke, the default bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TEST_TIMEOUT=900 BENCH_TIMEOUT=900 TAG=r06_final bash tools/gpu_steps.sh tests smoke bench
