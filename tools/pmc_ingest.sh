#!/bin/bash
# PMC passes (one counter group per run) over the ingest timing loop of one workload (tools/ablate.py).
# Usage: pmc_ingest.sh <workload> [group numbers]
W=${1:-cfg2}
SEL=${2:-"1 5"}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
G[1]="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
G[2]="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH"
G[5]="SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_ATOMIC_RETURN SQ_BUSY_CYCLES"
for i in $SEL; do
  timeout -s KILL 60 rocprofv3 --pmc ${G[$i]} --output-format csv -d "$R/gpurun_out/pmci_${W}_$i" -o run -- python3 "$R/tools/ablate.py" "$W" 0 > "$R/gpurun_out/pmci_${W}_$i.log" 2>&1 || { tail -5 "$R/gpurun_out/pmci_${W}_$i.log"; exit 1; }
done
