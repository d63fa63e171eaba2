cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
GS_PHASE_PROFILE=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 60 --warmup 20 > gpurun_out/phase_main.log 2>&1 || exit 1
tail -1 gpurun_out/phase_main.log
bash scripts/pmc.sh sq1:SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_VMEM sq2:SQ_INSTS_SALU,SQ_INSTS_FLAT,SQ_LDS_BANK_CONFLICT,SQ_LDS_ADDR_CONFLICT,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VMEM,SQ_INST_LEVEL_VMEM
