#!/bin/bash
# Two ranks on the box's one GPU (GS_BENCH_DEVICE=0): the driver's multi-GPU bench line
# (origin sharding of one network, with the one-engine check) and the C4 sweep workload.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03/mg
mkdir -p $OUT
GS_BENCH_DEVICE=0 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --check-shard > $OUT/c2_w2.log 2>&1 || { tail -5 $OUT/c2_w2.log; exit 1; }
grep '"metric"' $OUT/c2_w2.log | tail -1 > $OUT/c2_w2.json; cut -c1-700 $OUT/c2_w2.json
GS_BENCH_DEVICE=0 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 10 --warmup 5 --workload c4 > $OUT/c4_w2.log 2>&1 || { tail -5 $OUT/c4_w2.log; exit 1; }
grep '"metric"' $OUT/c4_w2.log | tail -1 > $OUT/c4_w2.json; cut -c1-900 $OUT/c4_w2.json
