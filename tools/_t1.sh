set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "key_row or varchar or composite" > gpurun_out/t1.log 2>&1; rc=$?
tail -15 gpurun_out/t1.log; exit $rc
