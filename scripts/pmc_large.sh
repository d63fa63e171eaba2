#!/bin/bash
# PMC passes over the bench's c4/c3 legs (one counter group per rocprofv3 run,
# --kernel-trace only). Output: gpurun_out/r02/pmc_large/<tag>/
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02/${PMC_DIR:-pmc_large}
mkdir -p $OUT
run() {  # run <tag> <counters...>
  local tag=$1; shift
  echo "== pmc $tag: $*"
  timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$tag -o run -- \
    python3 bench.py --only-large --large-mode ${LARGE_MODE:-4} --legs ${LEGS:-c4,c3} > $OUT/$tag.log 2>&1
  local rc=$?
  echo "== exit $rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$tag.log; exit $rc; fi
}
for spec in "${@}"; do
  tag=${spec%%:*}; ctrs=${spec#*:}
  run $tag ${ctrs//,/ }
done
