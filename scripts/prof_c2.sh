#!/bin/bash
# C2 alone (bench.py main leg, no large legs, no CPU baseline): rocprofv3 kernel-trace
# --stats, then one PMC pass per counter group (--kernel-trace only).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02/c2
mkdir -p $OUT
ARGS="--no-large --no-cpu-baseline --steps ${STEPS:-100} --warmup ${WARMUP:-20}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
grep -h '"metric"' $OUT/trace.log | tail -1 | cut -c1-400
for spec in "sq1:SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES" \
            "sq2:SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS,SQ_INSTS_SMEM" \
            "fetch:FETCH_SIZE" "write:WRITE_SIZE,TA_BUSY_avr,TA_TA_BUSY_sum"; do
  tag=${spec%%:*}; ctrs=${spec#*:}
  timeout -k 10 240 rocprofv3 --pmc ${ctrs//,/ } --kernel-trace --output-format csv -d $OUT/$tag -o run -- \
    python3 bench.py $ARGS > $OUT/$tag.log 2>&1 || { echo "pmc $tag failed"; tail -5 $OUT/$tag.log; exit 1; }
  echo "== pmc $tag ok"
done
