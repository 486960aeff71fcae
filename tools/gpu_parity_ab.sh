#!/bin/bash
# GPU box: the merge parity tests (every compiled layout, runs and cells), then bench A/B lines of
# $VARIANTS over $WLS (tools/ab_variants.sh).  Every GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compact_rows.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_parity.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_parity.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gpu_parity.log | head -20; exit $rc; }
bash tools/ab_variants.sh
