#!/bin/bash
# GPU box, end of a round: smoke + the full -m gpu suite, then tools/measure.sh (TAG), then the
# default bench line.  Every step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r06} PMC_WLS=${PMC_WLS:-"cfg2 cfg3 cfg4 cfg5 cfg4_10m"} BENCH_WLS=${BENCH_WLS:-"cfg2 cfg3 cfg4 cfg5 cfg4_10m"} bash tools/measure.sh > gpurun_out/measure.log 2>&1 || { tail -5 gpurun_out/measure.log; exit 1; }
echo measure ok
