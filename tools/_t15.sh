set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export FW_LIB_VARIANT=diag
for w in cfg5 cfg2; do
for ab in 0 1 2 4 6 7; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/abl_${w}_$ab -o run -- python3 $R/tools/ablate.py $w $ab > $R/gpurun_out/abl.log 2>&1 || { tail $R/gpurun_out/abl.log; exit 1; }
  python3 -c "
import csv,glob
f=glob.glob('$R/gpurun_out/abl_${w}_$ab/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'k_ingest' in r['Name']: print('$w', $ab, r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')
"
done
done
