#!/bin/bash
# k_ingest study on the GPU box: phase ablations (diagnostic build libflinkwin_diag.so) under each
# env in ENVS, then PMC groups (tools/pmc_ingest.sh) on the production build.
set -o pipefail
W=${W:-cfg2}
ENVS=${ENVS:-"FW_PACK=1"}
VARS=${VARS:-"0,1,4,6,7"}
mkdir -p gpurun_out
for e in $ENVS; do
  echo "== $e"
  ( export ${e//,/ }; FW_LIB_VARIANT=diag timeout -k 10 200 python -u tools/ablate.py "$W" "$VARS" ) 2>gpurun_out/abl_$W.err || { tail -5 gpurun_out/abl_$W.err; exit 1; }
done
if [ -n "$PMC" ]; then
  bash tools/pmc_ingest.sh "$W" "$PMC" || exit 1
  for g in $PMC; do python3 tools/pmc_sum.py gpurun_out/pmci_${W}_$g; done
fi
