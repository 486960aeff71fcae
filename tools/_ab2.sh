set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for w in ${WLS:-cfg2 cfg5}; do for nar in 0 1 0 1; do
FW_NARROW=$nar timeout -k 10 240 python bench.py --workload $w --no-cpu-baseline --no-e2e > gpurun_out/ab_$w.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/ab_$w.json'));r=d['roofline'];print('$w nar=$nar', round(d['value']/1e9,2), 'G ev/s', round(d['ms_per_step'],4), {k: round(v*1e3,1) for k,v in d['device_ms_per_step'].items()})"
done; done
