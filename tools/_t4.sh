set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for w in cfg2 cfg3; do for nar in 0 1; do
FW_NARROW=$nar timeout -k 10 240 python bench.py --workload $w --no-cpu-baseline --no-e2e > gpurun_out/b_$w.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b_$w.json'));r=d['roofline'];m=d['roofline_merge'];print('$w nar=$nar', round(d['value']/1e9,2), 'G ev/s', round(d['ms_per_step'],4), {k: round(v*1e3,1) for k,v in d['device_ms_per_step'].items()}, 'pbytes/launch', round(r['partial_bytes_written_per_launch']/1e6,1), 'compact', round(r['compact_chunk_share'],3))"
done; done
