#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT/profiles"
cd /tmp && export TMPDIR=/tmp
w=cfg4_10m
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$w" -o run -- python3 "$R/bench.py" --workload "$w" --steps 6 --warmup 1 --no-cpu-baseline --calibrate-traffic > "$OUT/pmc_fetch_$w.log" 2>&1 || { tail -20 "$OUT/pmc_fetch_$w.log"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$w" -o run -- python3 "$R/bench.py" --workload "$w" --steps 6 --warmup 1 --no-cpu-baseline --calibrate-traffic > "$OUT/pmc_write_$w.log" 2>&1 || { tail -20 "$OUT/pmc_write_$w.log"; exit 1; }
python3 "$R/tools/traffic.py" "$w" "$OUT/pmc_fetch_$w" "$OUT/pmc_write_$w" "$OUT/profiles/traffic_$w.json" || exit 1
timeout -k 10 240 python3 "$R/bench.py" --workload "$w" --no-cpu-baseline --traffic-json "$OUT/profiles/traffic_$w.json" > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail -20 "$OUT/bench_$w.err"; exit 1; }
