set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_compact_rows.py tests/test_gpu_parity.py -k "compact or async or two_phase or beyond or split or rescale" -q -x --timeout 120 --timeout-method thread -rs > gpurun_out/t_new.log 2>&1; rc=$?
tail -8 gpurun_out/t_new.log; [ $rc -eq 0 ] || exit $rc
for w in cfg2 cfg3 cfg4 cfg5; do
timeout -k 10 240 python bench.py --workload $w --no-cpu-baseline > gpurun_out/b_$w.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b_$w.json'));r=d['roofline'];m=d['roofline_merge'];e=d['end_to_end'];print('$w', round(d['value']/1e9,2), 'G ev/s', round(d['ms_per_step'],4), {k: round(v*1e3,1) for k,v in d['device_ms_per_step'].items()}, 'frac', round(r['frac'],3), round(m['frac'],3), 'pbytes/launch', round(r['partial_bytes_written_per_launch']/1e6,1), 'compact', round(r['compact_chunk_share'],3), 'e2e', round(e['value']/1e9,3))"
done
# N=2 rehearsal on one GPU (gloo, exchange staged through host memory): one-phase cfg2, two-phase cfg5
for w in cfg2 cfg5; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 6 --warmup 2 --workload $w --dist-backend gloo --no-cpu-baseline > gpurun_out/b2_$w.json 2> gpurun_out/b2.err || { tail -30 gpurun_out/b2.err; exit 1; }
python -c "import json;d=json.loads([l for l in open('gpurun_out/b2_$w.json') if l.startswith('{')][-1]);print('N=2 gloo $w', d['config']['plan'], round(d['value']/1e9,3), 'G ev/s', {k: round(v*1e3,1) for k,v in d['device_ms_per_step'].items()})"
done
