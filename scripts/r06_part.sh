#!/bin/bash
# Round 6: per-rank shares of the node-range partition on one GPU (scripts/part_share.py):
# K gloo ranks on device 0, engine calls serialized across ranks.
#   CASES="nodes:K:bfs[:backend] ..." (default: 1M x2 frontier, C5 x2 frontier, C5 x2 replicated)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r06/${TAG:-part}
mkdir -p $OUT
CASES=${CASES:-"1000000:2:frontier 10000000:2:frontier 10000000:2:replicated"}
port=29611
for c in $CASES; do
  IFS=: read -r n k bfs be <<< "$c"
  port=$((port + 1))
  echo "== $n nodes, $k ranks, $bfs"
  timeout -k 10 ${CASE_TO:-500} python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $k --master-addr 127.0.0.1 \
    --master-port $port scripts/part_share.py --nodes $n --bfs $bfs --backend ${be:-gloo} ${ARGS:-} > $OUT/part_${n}_${k}_${bfs}${be}.log 2>&1 \
    || { tail -20 $OUT/part_${n}_${k}_${bfs}${be}.log; exit 1; }
  grep '^{' $OUT/part_${n}_${k}_${bfs}${be}.log
done
