#!/bin/bash
# Round 4: two ranks on the box's one GPU (GS_BENCH_DEVICE=0), the driver's launch line:
# the default C2 bench (weak: rank r = trial r), C2 strong with the one-engine shard check,
# C4 weak / strong and C5 strong (origin sharding). These rehearse launch, rendezvous,
# sharding and assembly; with both ranks on one device they say nothing about scaling.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04/mg
mkdir -p $OUT
run() {  # run <tag> <port> <bench args...>
  local tag=$1 port=$2; shift 2
  echo "== $tag"
  GS_BENCH_DEVICE=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 "$@" > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
  grep '"metric"' $OUT/$tag.log | tail -1 > $OUT/$tag.json
  python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print(d['scaling'], d['value'], round(d['ms_per_step'],3), d['config'].get('parallelism'), d.get('shard_check'))"
}
run c2_weak 29541 --steps 20 --warmup 5 --no-cpu-baseline --no-large
run c2_strong 29542 --steps 20 --warmup 5 --scaling strong --check-shard
run c4_weak 29543 --steps 10 --warmup 5 --workload c4
run c4_strong 29544 --steps 10 --warmup 5 --workload c4 --scaling strong
run c5_strong 29545 --steps 5 --warmup 3 --workload c5 --scaling strong
