#!/bin/bash
# Instruction-cache PMC pass over the ingest timing loop and the merge loop of one workload.
W=${1:-cfg2}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d "$R/gpurun_out/pmcic_${W}_i" -o run -- python3 "$R/tools/ablate.py" "$W" 0 > "$R/gpurun_out/pmcic_${W}_i.log" 2>&1 || { tail -5 "$R/gpurun_out/pmcic_${W}_i.log"; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d "$R/gpurun_out/pmcic_${W}_m" -o run -- python3 "$R/tools/ablate.py" merge "$W" 0 > "$R/gpurun_out/pmcic_${W}_m.log" 2>&1 || { tail -5 "$R/gpurun_out/pmcic_${W}_m.log"; exit 1; }
