#!/bin/bash
# A/B of library variants (gossip-sim_amd/variants/<v>/libgossip_hip.so; "" = the in-tree
# build) on the C2 driver window and the prune-wave round (round 19 alone), interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03/${TAG:-var}
mkdir -p $OUT
for rep in 1 2; do
  for v in "$@"; do
    lab=${v:-head}
    [ "$v" = head ] && v=""
    GS_LIB_VARIANT=$v timeout -k 10 200 python3 bench.py --no-large --no-cpu-baseline --no-steady --steps 20 --warmup 5 > $OUT/c2_$lab.json 2>&1 || { tail -5 $OUT/c2_$lab.json; exit 1; }
    GS_LIB_VARIANT=$v timeout -k 10 200 python3 bench.py --no-large --no-cpu-baseline --no-steady --steps 1 --warmup 19 > $OUT/w_$lab.json 2>&1 || { tail -5 $OUT/w_$lab.json; exit 1; }
    GS_LIB_VARIANT=$v timeout -k 10 200 python3 bench.py --no-large --no-cpu-baseline --no-steady --steps 100 --warmup 60 > $OUT/s_$lab.json 2>&1 || { tail -5 $OUT/s_$lab.json; exit 1; }
    echo "$lab rep $rep: window $(grep -o '"avg_launch_us": [0-9.]*' $OUT/c2_$lab.json | head -1)  wave $(grep -o '"avg_launch_us": [0-9.]*' $OUT/w_$lab.json | head -1)  steady $(grep -o '"avg_launch_us": [0-9.]*' $OUT/s_$lab.json | head -1)"
  done
done
