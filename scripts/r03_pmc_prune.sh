#!/bin/bash
# PMC passes over the c4 leg; per-dispatch counters of the prune wave's k_cg_prune.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r03/pmc_prune
mkdir -p $OUT
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "FETCH_SIZE TA_BUSY_avr" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU TA_TA_BUSY_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
    python3 bench.py --only-large --legs c4 > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/pmc_disp.py ${KERN:-k_cg_prune} ${RANK:-SQ_WAVE_CYCLES} $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4 > $OUT/summary.txt; cat $OUT/summary.txt
