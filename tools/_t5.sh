set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # variant narrow workload
  if [ "$1" = default ]; then unset FW_LIB_VARIANT; else export FW_LIB_VARIANT=$1; fi
  FW_NARROW=$2 timeout -k 10 240 python bench.py --workload $3 --no-cpu-baseline --no-e2e > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$3 $1 nar=$2', round(d['value']/1e9,2), 'G ev/s', {k: round(v*1e3,1) for k,v in d['device_ms_per_step'].items()})"
}
for w in cfg2 cfg5; do
  run default 0 $w; run nb 0 $w; run default 1 $w; run default 0 $w; run nb 0 $w; run default 1 $w
done
unset FW_LIB_VARIANT
FW_LIB_VARIANT=diag timeout -k 10 240 python tools/ablate.py merge cfg2 0,128 > gpurun_out/diag_cfg2.log 2>&1 || { tail gpurun_out/diag_cfg2.log; exit 1; }
cat gpurun_out/diag_cfg2.log
