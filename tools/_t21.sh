set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # variant workload
  if [ "$1" = default ]; then unset FW_LIB_VARIANT; else export FW_LIB_VARIANT=$1; fi
  timeout -k 10 200 python bench.py --workload $2 --no-cpu-baseline --no-e2e > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$2 $1', round(d['value']/1e9,2), 'G ev/s', round(d['ms_per_step']*1e3,1), 'us', {k: round(v*1e3,1) for k,v in d['device_ms_per_step'].items()})"
}
for w in cfg2 cfg3; do run base $w; run p1 $w; run base $w; run p1 $w; done
for w in cfg5; do run base $w; run default $w; done
export FW_LIB_VARIANT=p1
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_p1.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests_p1.log
unset FW_LIB_VARIANT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc2=$?
tail -2 gpurun_out/gpu_tests.log; exit $(( rc || rc2 ))
