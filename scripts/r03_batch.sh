#!/bin/bash
# Round 3 batch: parity tests touching the gs_round consume/prune kernels, the c4 leg A/B
# against the previous prune kernel (with the prune-wave round's time), 2-rank rehearsals.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r03/batch
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_partition.py tests/test_cli.py -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  -k "fused_round_matches_steps or simulation_parity_c1 or simulation_stats or c4_sweep or small-gloo or cli_run" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log
if [ $rc -ne 0 ]; then grep -m5 -B2 -A30 "Error\|assert" $OUT/tests.log | head -60; exit $rc; fi
for rep in 1 2; do
  for v in head oldprune; do
    vv=$v; [ "$v" = head ] && vv=""
    GS_LIB_VARIANT=$vv timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_$v -o run -- python3 bench.py --only-large --legs c4 > $OUT/c4_$v.json 2>&1 || { tail -5 $OUT/c4_$v.json; exit 1; }
    echo "$v rep $rep: $(grep -o '"ms_per_step": [0-9.]*' $OUT/c4_$v.json) wave-round prune: $(python3 scripts/launch_times.py $OUT/tr_$v k_cg_prune | tr ' ' '\n' | sort -n | tail -1) us"
  done
done
GS_BENCH_DEVICE=0 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --check-shard > $OUT/c2_w2.log 2>&1 || { tail -5 $OUT/c2_w2.log; exit 1; }
grep '"metric"' $OUT/c2_w2.log | cut -c1-600
GS_BENCH_DEVICE=0 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 10 --warmup 5 --workload c4 > $OUT/c4_w2.log 2>&1 || { tail -5 $OUT/c4_w2.log; exit 1; }
grep '"metric"' $OUT/c4_w2.log | cut -c1-800
