set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES --output-format csv -d $R/gpurun_out/pmc_ig1 -o run -- python3 $R/tools/ablate.py cfg2 0 > $R/gpurun_out/pmc_ig1.log 2>&1 || { tail $R/gpurun_out/pmc_ig1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT --output-format csv -d $R/gpurun_out/pmc_ig2 -o run -- python3 $R/tools/ablate.py cfg2 0 > $R/gpurun_out/pmc_ig2.log 2>&1 || { tail $R/gpurun_out/pmc_ig2.log; exit 1; }
find $R/gpurun_out/pmc_ig1 $R/gpurun_out/pmc_ig2 -name "*counter_collection.csv" | head
