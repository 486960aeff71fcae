set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_compact_rows.py tests/test_gpu_parity.py -k "compact or async" -q -x --timeout 120 --timeout-method thread > gpurun_out/t_compact.log 2>&1; rc=$?
tail -15 gpurun_out/t_compact.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for w in cfg2 cfg3 cfg4 cfg5; do
timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > gpurun_out/b_$w.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b_$w.json'));r=d['roofline'];m=d['roofline_merge'];e=d['end_to_end'];print('$w', round(d['value']/1e9,2), 'G ev/s', round(d['ms_per_step'],4), {k: round(v*1e3,1) for k,v in d['device_ms_per_step'].items()}, 'frac', round(r['frac'],3), round(m['frac'],3), 'pbytes/launch', round(r['partial_bytes_written_per_launch']/1e6,1), 'compact', round(r['compact_chunk_share'],3), 'e2e', round(e['value']/1e9,3), {k: round(v,2) for k,v in e['host_ms_per_step'].items()}, round(e['fill_GBps'],1))"
done
