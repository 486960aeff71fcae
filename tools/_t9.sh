set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_heap_key_group.py tests/test_gpu_compact_rows.py -v -x --timeout 200 --timeout-method thread > gpurun_out/heap_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error" gpurun_out/heap_tests.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --workload cfg2 --no-cpu-baseline > gpurun_out/b_cfg2.json 2> gpurun_out/b_cfg2.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/b_cfg2.json'));print(d['value']/1e9, d['end_to_end'])"
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; exit $rc
