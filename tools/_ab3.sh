set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # variant skip workload
  if [ "$1" = default ]; then unset FW_LIB_VARIANT; else export FW_LIB_VARIANT=$1; fi
  FW_SKIP_IDLE=$2 timeout -k 10 240 python bench.py --workload $3 --no-cpu-baseline --no-e2e > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$3 $1 skip=$2', round(d['value']/1e9,2), 'G ev/s', round(d['ms_per_step']*1e3,1), 'us', {k: round(v*1e3,1) for k,v in d['device_ms_per_step'].items()}, d['roofline_merge']['launches'])"
}
for w in cfg2 cfg3 cfg5; do
  run default 1 $w; run r0 1 $w; run default 0 $w; run default 1 $w; run r0 1 $w; run default 0 $w
done
export FW_LIB_VARIANT=
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; exit $rc
