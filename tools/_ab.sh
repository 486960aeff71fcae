# A/B of library variants: VARS="'' p1" WLS="cfg2 cfg3" bash tools/_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for w in ${WLS:-cfg2 cfg3}; do for v in ${VARS:-default p1}; do
if [ "$v" = default ]; then unset FW_LIB_VARIANT; else export FW_LIB_VARIANT=$v; fi
timeout -k 10 240 python bench.py --workload $w --no-cpu-baseline --no-e2e > gpurun_out/ab_$w.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/ab_$w.json'));r=d['roofline'];print('$w $v', round(d['value']/1e9,2), 'G ev/s', round(d['ms_per_step'],4), {k: round(v*1e3,1) for k,v in d['device_ms_per_step'].items()})"
done; done
