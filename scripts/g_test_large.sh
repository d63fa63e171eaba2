cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest6.log 2>&1; rc=$?
tail -15 gpurun_out/pytest6.log
[ $rc -ne 0 ] && exit $rc
bash scripts/large_bench.sh
