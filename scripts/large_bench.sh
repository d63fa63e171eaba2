cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --nodes 100000 --slots 16 --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/b100k.log 2>&1 || { tail -20 gpurun_out/b100k.log; exit 1; }
tail -1 gpurun_out/b100k.log
timeout -k 10 400 python bench.py --nodes 1000000 --slots 8 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b1m.log 2>&1 || { tail -20 gpurun_out/b1m.log; exit 1; }
tail -1 gpurun_out/b1m.log
