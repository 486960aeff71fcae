set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  timeout -k 10 200 python bench.py --workload $1 --no-cpu-baseline --no-e2e > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$1 ev=${_AB_EVENTS:-0}', round(d['value']/1e9,2), 'G ev/s', round(d['ms_per_step']*1e3,1), 'us', {k: round(v*1e3,1) for k,v in d['device_ms_per_step'].items()}, 'issue', round(d['host_issue_ms_per_step']*1e3,1))"
}
for w in cfg2 cfg3 cfg5; do
  export _AB_EVENTS=1; run $w; unset _AB_EVENTS; run $w; export _AB_EVENTS=1; run $w; unset _AB_EVENTS; run $w
done
