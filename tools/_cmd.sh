set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -x > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -30 gpurun_out/gpu_tests.log
exit $rc
