set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_heap_key_group.py tests/test_gpu_key_rows.py -q -x --timeout 200 --timeout-method thread -k "heap or rescale" > gpurun_out/t18.log 2>&1; rc=$?
tail -15 gpurun_out/t18.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; exit $rc
