set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 180 --timeout-method thread -x -k "golden or random_stream or hot_keys or ltz" > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
b() { timeout -k 10 200 python bench.py --workload $1 --no-cpu-baseline --no-e2e > gpurun_out/b.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$1 $2', round(d['value']/1e9,2), 'G ev/s', round(d['ms_per_step'],4), {k: round(v*1e3,1) for k,v in d['device_ms_per_step'].items()}, 'sb', d['config']['superbuckets'], 'frac', round(d['roofline']['frac'],3), round(d['roofline_merge']['frac'],3))"; }
for w in cfg2 cfg3 cfg4 cfg5; do b $w; done
