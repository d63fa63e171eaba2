#!/bin/bash
# FETCH/WRITE per dispatch of the binned BFS kernels at 1M x 8 (2 steps).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export BENCH_ARGS="--nodes 1000000 --slots 8 --steps 2 --warmup 1 --bfs-mode 3 --no-cpu-baseline --no-profile"
bash scripts/pmc.sh lfetch:FETCH_SIZE lwrite:WRITE_SIZE
