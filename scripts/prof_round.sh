#!/bin/bash
# Phase profile + kernel-trace per-launch durations of the C2 bench, in one GPU call.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
GS_PHASE_PROFILE=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 60 --warmup 20 > gpurun_out/phase_main.log 2>&1 || exit 1
tail -1 gpurun_out/phase_main.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 60 --warmup 20 --no-cpu-baseline --no-profile > gpurun_out/rocprof.log 2>&1 || exit 1
python3 scripts/launch_times.py gpurun_out/prof k_round_wg
