#!/bin/bash
# Instruction counts of k_ingest per ablation variant (diagnostic build): one PMC pass per variant.
W=${W:-cfg2}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for ab in ${VARS:-0 4 6 32768}; do
  export FW_LIB_VARIANT=diag; timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d "$R/gpurun_out/pmcp_$ab" -o run -- python3 "$R/tools/ablate.py" "$W" "$ab" > "$R/gpurun_out/pmcp_$ab.log" 2>&1 || { tail -5 "$R/gpurun_out/pmcp_$ab.log"; exit 1; }
  echo "== ablate $ab"; python3 "$R/tools/pmc_sum.py" "$R/gpurun_out/pmcp_$ab" | grep k_ingest
done
