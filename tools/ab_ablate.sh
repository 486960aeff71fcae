#!/bin/bash
# merge-kernel phase attribution (diagnostic build, make DIAG=1 OUT=../libflinkwin_diag.so
# OBJDIR=build_diag): the bench's merge launch time with phases switched off (FW_ABLATE bits,
# fw_internal.h AB_M_*).  Results are meaningless under ablation; only kernel times matter.
#   WLS="cfg2" ABL="0 8 16 32 64 120" EXTRA="FW_RUNS=0" tools/ab_ablate.sh
set -o pipefail
OUT=${OUT:-gpurun_out}
WLS=${WLS:-cfg2}
ABL=${ABL:-"0 8 16 32 64 4096 120"}
mkdir -p "$OUT"
for w in $WLS; do
  for ab in $ABL; do
    timeout -k 10 200 env FW_LIB_VARIANT=diag FW_ABLATE=$ab $EXTRA python -u bench.py --workload "$w" --steps 24 --no-cpu-baseline --no-e2e > "$OUT/abl_${w}_$ab.json" 2> "$OUT/abl_${w}_$ab.err" || { tail -5 "$OUT/abl_${w}_$ab.err"; continue; }
    python3 -c "import json;d=json.load(open('$OUT/abl_${w}_$ab.json'));print('$w ablate=$ab $EXTRA', 'merge_us', round(d['roofline_merge']['avg_launch_us'] or 0,1), 'launches', d['roofline_merge']['launches'], 'ingest_us', round(d['roofline']['avg_launch_us'],1))"
  done
done
