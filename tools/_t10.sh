set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --workload cfg2 --no-cpu-baseline > gpurun_out/b_cfg2.json 2> gpurun_out/b_cfg2.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/b_cfg2.json'));print(d['value']/1e9, d['end_to_end'])"
export FW_LIB_VARIANT=diag
for w in cfg2 cfg5; do timeout -k 10 120 python tools/ablate.py $w 0,2,4,6 || exit 1; done
