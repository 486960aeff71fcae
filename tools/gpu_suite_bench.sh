#!/bin/bash
# GPU box: the full -m gpu suite, then short bench lines (WLS, default cfg4_10m cfg2 cfg5):
#   bash tools/gpu_suite_bench.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gpu_tests.log | head -20; exit $rc; }
for w in ${WLS:-cfg4_10m cfg2 cfg5}; do
  timeout -k 10 200 python -u bench.py --workload $w --steps 24 --no-cpu-baseline --no-e2e > gpurun_out/p3_$w.json 2> gpurun_out/p3_$w.err || { tail -5 gpurun_out/p3_$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/p3_$w.json'));print('$w', round(d['value']/1e9,2),'G ev/s', 'merge_us', round(d['roofline_merge']['avg_launch_us'] or 0,1), 'ingest_us', round(d['roofline']['avg_launch_us'],1))"
done
