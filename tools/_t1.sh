set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "datastream or ds_ or golden or nan or full_size" > gpurun_out/t1.log 2>&1; rc=$?
tail -15 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
cat gpurun_out/b.json
