#!/bin/bash
# A/B of one environment switch of the library on the GPU box (run through gpurun from the repo root):
#   AB="FW_RUNS=0" WLS="cfg2 cfg3" tools/ab_env.sh
# runs each workload's bench line with and without the switch (alternating, REPS times), then
# prints events/s and the per-kernel device time per step.  Every GPU step has its own time limit.
set -o pipefail
OUT=${OUT:-gpurun_out}
WLS=${WLS:-"cfg2 cfg3 cfg4 cfg5"}
REPS=${REPS:-1}
STEPS=${STEPS:-24}
mkdir -p "$OUT"
one() {  # label env workload
  timeout -k 10 200 env $2 python -u bench.py --workload "$3" --steps "$STEPS" --no-cpu-baseline --no-e2e > "$OUT/ab_$3_$1.json" 2> "$OUT/ab_$3_$1.err" || { tail -20 "$OUT/ab_$3_$1.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/ab_$3_$1.json'));print('$3 $1', round(d['value']/1e9,2), 'G ev/s', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v*1e3,1) for k,v in d['device_ms_per_step'].items()}, 'merge_us', round(d['roofline_merge']['avg_launch_us'] or 0,1), 'ingest_us', round(d['roofline']['avg_launch_us'],1))"
}
for r in $(seq $REPS); do
  for w in $WLS; do
    one base "FW_AB_BASE=1 $AB" "$w" || exit 1
    one new "FW_AB_NEW=1" "$w" || exit 1
  done
done
