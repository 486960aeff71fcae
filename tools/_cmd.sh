set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "two_phase" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests2.log 2>&1; rc=$?; tail -5 gpurun_out/gpu_tests2.log; [ $rc -eq 0 ] || exit $rc
for w in cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-e2e > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { tail gpurun_out/bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));print('$w', round(d['value']/1e9,2), 'G ev/s', d['device_ms_per_step'], 'ingest frac', round(d['roofline']['frac'],3), 'merge frac', round(d['roofline_merge']['frac'],3))"
done
