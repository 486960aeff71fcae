set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "hop or HOP or golden or rescale or layouts or ltz or composite or varchar or two_phase or split" > gpurun_out/t1.log 2>&1; rc=$?
tail -15 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
for w in cfg3 cfg2; do
timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-e2e > gpurun_out/b_$w.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b_$w.json'));print('$w', round(d['value']/1e9,2), 'G ev/s', round(d['ms_per_step'],4), {k: round(v*1e3,1) for k,v in d['device_ms_per_step'].items()}, 'sb', d['config']['superbuckets'], 'frac', round(d['roofline']['frac'],3), round(d['roofline_merge']['frac'],3))"
done
