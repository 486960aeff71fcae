#!/bin/bash
# GPU-box check used during development (run through gpurun from the repo root):
#   parity tests, then one bench line per workload, then a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out}
STEPS=${STEPS:-24}
WLS=${WLS:-"cfg2 cfg3 cfg4 cfg5"}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
for w in $WLS; do
  timeout -k 10 240 python -u bench.py --workload "$w" --steps "$STEPS" --warmup 3 --no-cpu-baseline > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail -20 "$OUT/bench_$w.err"; exit 1; }
  cat "$OUT/bench_$w.json"
done
if [ -n "$PROF" ]; then
  R=$GRAFT_REPO_ROOT
  cd /tmp && export TMPDIR=/tmp
  for w in $PROF; do
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_$w" -o run -- python3 "$R/bench.py" --workload "$w" --steps "$STEPS" --warmup 3 --no-cpu-baseline > "$R/$OUT/prof_$w.log" 2>&1 || { tail -20 "$R/$OUT/prof_$w.log"; exit 1; }
  done
fi
