#!/bin/bash
# PMC passes (one counter group per run) over the merge ablation loop of one workload.
# Usage: pmc_merge.sh <workload> [group numbers, default all]
W=${1:-cfg3}
SEL=${2:-"1 2 3 4"}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
G[1]="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
G[2]="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH"
G[3]="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"
G[5]="SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_ATOMIC_RETURN SQ_BUSY_CYCLES"
G[6]="SQ_LDS_IDX_ACTIVE SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_WAVE_CYCLES"
G[4]="TCC_HIT_sum TCC_MISS_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_STALL_MULTI_MISS_sum"
for i in $SEL; do
  timeout -s KILL 60 rocprofv3 --pmc ${G[$i]} --output-format csv -d "$R/gpurun_out/pmc_${W}_$i" -o run -- python3 "$R/tools/ablate.py" merge "$W" ${AB:-0} > "$R/gpurun_out/pmc_${W}_$i.log" 2>&1 || { tail -5 "$R/gpurun_out/pmc_${W}_$i.log"; exit 1; }
done
