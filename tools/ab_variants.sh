#!/bin/bash
# bench lines of several library builds / environment switches on the GPU box (run through gpurun):
#   VARIANTS="base:FW_RUNS=0 new: g3:FW_LIB_VARIANT=g3" WLS="cfg2 cfg4" tools/ab_variants.sh
# each variant is label:ENV=VAL[,ENV=VAL...]; prints events/s and per-kernel device time per step.
set -o pipefail
OUT=${OUT:-gpurun_out}
WLS=${WLS:-cfg2}
REPS=${REPS:-1}
STEPS=${STEPS:-24}
mkdir -p "$OUT"
for r in $(seq $REPS); do
  for w in $WLS; do
    for v in $VARIANTS; do
      lab=${v%%:*}; envs=${v#*:}; envs=${envs//,/ }
      timeout -k 10 200 env FW_AB=1 $envs python -u bench.py --workload "$w" --steps "$STEPS" --no-cpu-baseline --no-e2e > "$OUT/ab_${w}_$lab.json" 2> "$OUT/ab_${w}_$lab.err" || { tail -20 "$OUT/ab_${w}_$lab.err"; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/ab_${w}_$lab.json'));print('$w $lab', round(d['value']/1e9,2), 'G ev/s', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v*1e3,1) for k,v in d['device_ms_per_step'].items()}, 'merge_us', round(d['roofline_merge']['avg_launch_us'] or 0,1), 'ingest_us', round(d['roofline']['avg_launch_us'],1))"
    done
  done
done
