#!/bin/bash
# GPU box: rocprofv3 kernel trace of one rank through bench.py's N > 1 path over RCCL (cfg2)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
W=${W:-cfg2}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_rccl" -o run \
  -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29515 \
  "$R/bench.py" --gpus 1 --dist-backend nccl --force-collectives --workload $W --no-cpu-baseline --steps 12 --warmup 2 \
  > "$R/gpurun_out/prof_rccl.json" 2> "$R/gpurun_out/prof_rccl.err" || { tail -20 "$R/gpurun_out/prof_rccl.err"; exit 1; }
python3 - "$R/gpurun_out/prof_rccl" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)
for r in list(csv.DictReader(open(f[0])))[:25]:
    print("%-90s %6s %10.1f us avg %8.1f ms total" % (r["Name"][:90], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
