set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # variant workload
  if [ "$1" = default ]; then unset FW_LIB_VARIANT; else export FW_LIB_VARIANT=$1; fi
  timeout -k 10 240 python bench.py --workload $2 --no-cpu-baseline --no-e2e > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$2 $1', round(d['value']/1e9,2), 'G ev/s', {k: round(v*1e3,1) for k,v in d['device_ms_per_step'].items()})"
}
for w in cfg2 cfg3 cfg4 cfg5; do run default $w; run w8 $w; run default $w; run w8 $w; done
export FW_LIB_VARIANT=w8
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "random_stream or layouts or golden or compact or hop" > gpurun_out/t_w8.log 2>&1; rc=$?
tail -3 gpurun_out/t_w8.log; exit $rc
