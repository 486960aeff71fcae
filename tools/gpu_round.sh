#!/bin/bash
# GPU-box check of a development step: the -m gpu suite, then (if green) one default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
timeout -k 10 ${TEST_TIMEOUT:-840} python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 300 --timeout-method thread \
  ${PYTEST_ARGS:-} > "$OUT/gpu_tests.log" 2>&1
rc=$?
tail -40 "$OUT/gpu_tests.log"
[ $rc -eq 0 ] || exit $rc
[ -n "${SKIP_BENCH:-}" ] && exit 0
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
