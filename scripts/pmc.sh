#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only, no
# tracing domains) over a short bench run. Output: gpurun_out/pmc/<tag>/...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
ARGS=${BENCH_ARGS:-"--steps 20 --warmup 22 --no-cpu-baseline --no-profile --no-large"}
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
run() {  # run <tag> <counters...>
  local tag=$1; shift
  echo "== pmc $tag: $*"
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc/$tag -o run -- python3 bench.py $ARGS > gpurun_out/pmc/$tag.log 2>&1
  local rc=$?
  echo "== exit $rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/$tag.log; exit $rc; fi
}
for spec in "${@}"; do
  tag=${spec%%:*}; ctrs=${spec#*:}
  run $tag $ctrs
done
