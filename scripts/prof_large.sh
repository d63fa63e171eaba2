#!/bin/bash
# rocprofv3 kernel trace of the large-N bench (per-level kernel durations).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in ${MODES:-2 3}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/proflarge_$m -o run -- \
    python3 bench.py --nodes ${NODES:-1000000} --slots ${SLOTS:-8} --steps 3 --warmup 2 --bfs-mode $m --no-cpu-baseline --no-profile --no-large \
    > gpurun_out/proflarge_$m.log 2>&1 || { echo "mode $m failed"; tail gpurun_out/proflarge_$m.log; exit 1; }
done
