set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/gpu_tests.log | head -20; exit $rc; }
VARIANTS="base:FW_RUNS=0 new:FW_X=1 g3:FW_LIB_VARIANT=g3 g4:FW_LIB_VARIANT=g4" WLS="cfg2 cfg4" tools/ab_variants.sh || exit 1
for r in 0 1; do FW_RUNS=$r FW_LIB_VARIANT=diag timeout -k 10 120 python -u tools/ablate.py cfg2 0,4,1 2>/dev/null | sed "s/^/runs=$r /" || exit 1; done
