#!/bin/bash
# GPU box: the parity tests of both partial-row layouts, then runs-vs-cells bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compact_rows.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_parity.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_parity.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gpu_parity.log | head -20; exit $rc; }
VARIANTS="planned:FW_X=1 cells:FW_RUNS=0" WLS="${WLS:-cfg4_10m cfg4 cfg2}" bash tools/ab_variants.sh
