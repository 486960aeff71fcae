#!/bin/bash
# PMC passes (one counter group per run) over the merge ablation loop of one workload.
W=${1:-cfg3}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "$R/gpurun_out/pmc_${W}_$i" -o run -- python3 "$R/tools/ablate.py" merge "$W" 0 > "$R/gpurun_out/pmc_${W}_$i.log" 2>&1 || { tail -5 "$R/gpurun_out/pmc_${W}_$i.log"; exit 1; }
done
