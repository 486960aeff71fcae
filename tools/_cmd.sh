set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_key_rows.py -q -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for w in cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-e2e > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { tail gpurun_out/bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));print('$w', round(d['value']/1e9,2), 'G ev/s', round(d['ms_per_step'],4), d['device_ms_per_step'], 'ingest frac', round(d['roofline']['frac'],3), 'merge frac', round(d['roofline_merge']['frac'],3))"
done
timeout -k 10 200 python tools/ablate.py merge cfg2 384 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python tools/ablate.py merge cfg3 384 2>&1 | grep -v amdgpu.ids
