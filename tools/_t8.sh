set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -rs > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -6 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
TAG=r03 PMC_WLS="cfg2 cfg3 cfg4 cfg5" BENCH_WLS="cfg2 cfg3 cfg4 cfg5 cfg4_10m" bash tools/measure.sh > gpurun_out/measure.log 2>&1; rc=$?
tail -3 gpurun_out/measure.log; exit $rc
