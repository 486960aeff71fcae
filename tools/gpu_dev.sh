#!/bin/bash
# Development check on the GPU box (through gpurun, repo root): optional parity tests, then bench
# lines per (env, workload) with a one-line summary each.  Every GPU step has its own time limit and
# the chain stops at the first failure.
#   TESTS="-k runs" (pytest args, empty: skip)  WLS="cfg2"  ENVS="FW_PACK=0 FW_PACK=1"  STEPS=20
set -o pipefail
OUT=${OUT:-gpurun_out}
STEPS=${STEPS:-20}
WLS=${WLS:-"cfg2"}
ENVS=${ENVS:-"-"}
mkdir -p "$OUT"
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $TESTS > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
  tail -2 "$OUT/gpu_tests.log"
fi
for e in $ENVS; do
  for w in $WLS; do
    tag=$(echo "$e" | tr '=,' '__')_$w
    ( [ "$e" != "-" ] && export ${e//,/ }; timeout -k 10 240 python -u bench.py --workload "$w" --steps "$STEPS" --warmup 3 --no-cpu-baseline ${BENCH_ARGS} ) > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || { tail -20 "$OUT/bench_$tag.err"; exit 1; }
    python3 tools/summ.py "$e" "$OUT/bench_$tag.json"
  done
done
