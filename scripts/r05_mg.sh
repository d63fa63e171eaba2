#!/bin/bash
# Round 5: two ranks on the box's one GPU (GS_BENCH_DEVICE=0) with the driver's launch line:
# the C2 default (origin-split strong scaling) with the one-engine check and the weak_trial
# key, and the C3 sweep workload (16 sims dealt round-robin). They rehearse launch,
# rendezvous, sharding and assembly; both ranks share one device, so not scaling.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05/mg
P=gpurun_out/r05/mg  # (copied into profiles/r05/mg/ after the call)
mkdir -p $OUT $P
GS_BENCH_DEVICE=0 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 2 --steps 20 --warmup 5 --check-shard > $OUT/c2_w2.log 2>&1 || { tail -5 $OUT/c2_w2.log; exit 1; }
grep '"metric"' $OUT/c2_w2.log | tail -1 > $P/c2_w2.json; cut -c1-300 $P/c2_w2.json; echo
python3 -c "import json; d=json.load(open('$P/c2_w2.json')); print('shard_check', d.get('shard_check'), 'weak_trial', d.get('weak_trial'))"
GS_BENCH_DEVICE=0 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 2 --steps 20 --warmup 5 --workload c3 > $OUT/c3_w2.log 2>&1 || { tail -5 $OUT/c3_w2.log; exit 1; }
grep '"metric"' $OUT/c3_w2.log | tail -1 > $P/c3_w2.json; cut -c1-600 $P/c3_w2.json; echo
