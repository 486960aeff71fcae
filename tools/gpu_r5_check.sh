#!/bin/bash
# GPU box (round 5): the whole GPU test suite on the default library, then bench A/B lines of
# $VARIANTS over $WLS (tools/ab_variants.sh).  Every GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r5_tests.log | head -20; exit $rc; }
[ -z "$VARIANTS" ] || bash tools/ab_variants.sh
