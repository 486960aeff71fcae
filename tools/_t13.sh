set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -s KILL 120 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 --output-format csv -d $R/gpurun_out/pcs -o run -- python3 $R/tools/ablate.py cfg2 0 > $R/gpurun_out/pcs.log 2>&1 || { tail -20 $R/gpurun_out/pcs.log; exit 1; }
ls -la $R/gpurun_out/pcs/ ; tail -3 $R/gpurun_out/pcs.log
