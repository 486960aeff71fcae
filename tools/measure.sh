#!/bin/bash
# Round measurement on the GPU box (run through gpurun from the repo root):
#   1. the default bench line (cfg2, with the CPU baseline leg) under rocprofv3 --kernel-trace --stats
#   2. per workload in $PMC_WLS: FETCH_SIZE and WRITE_SIZE passes (separate runs) + tools/traffic.py
#   3. plain bench lines of the other workloads (traffic file from step 2 picked up)
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${TAG:-r01}
PMC_WLS=${PMC_WLS:-"cfg2"}
BENCH_WLS=${BENCH_WLS:-"cfg2 cfg3 cfg4 cfg5"}
mkdir -p "$OUT/profiles"
cd /tmp && export TMPDIR=/tmp
if [ -z "$SKIP_DEFAULT" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_default" -o run \
  -- python3 "$R/bench.py" > "$OUT/bench_default.json" 2> "$OUT/prof_default.log" || { tail -20 "$OUT/prof_default.log"; exit 1; }
cat "$OUT/bench_default.json"
fi
for w in $PMC_WLS; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$w" -o run \
    -- python3 "$R/bench.py" --workload "$w" --steps 6 --warmup 1 --no-cpu-baseline --calibrate-traffic > "$OUT/pmc_fetch_$w.log" 2>&1 || { tail -20 "$OUT/pmc_fetch_$w.log"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$w" -o run \
    -- python3 "$R/bench.py" --workload "$w" --steps 6 --warmup 1 --no-cpu-baseline --calibrate-traffic > "$OUT/pmc_write_$w.log" 2>&1 || { tail -20 "$OUT/pmc_write_$w.log"; exit 1; }
  python3 "$R/tools/traffic.py" "$w" "$OUT/pmc_fetch_$w" "$OUT/pmc_write_$w" "$OUT/profiles/traffic_$w.json" || exit 1
done
for w in $BENCH_WLS; do
  timeout -k 10 240 python3 "$R/bench.py" --workload "$w" --no-cpu-baseline \
    --traffic-json "$OUT/profiles/traffic_$w.json" > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail -20 "$OUT/bench_$w.err"; exit 1; }
  cat "$OUT/bench_$w.json"
done
