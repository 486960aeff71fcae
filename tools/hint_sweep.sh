#!/bin/bash
# Capacity-hint sweep: bench lines of WL workloads at each state_per_key hint (0 = the workload's own),
# without the end-to-end and CPU legs; peak superbucket entries against the table capacity in each line.
set -e
OUT=${OUT:-gpurun_out/hint}
mkdir -p "$OUT"
for wl in ${WLS:-cfg4_10m}; do
  for h in ${HINTS:-0}; do
    extra=""
    [ "$h" != "0" ] && extra="--state-per-key $h"
    timeout -k 10 240 python -u bench.py --workload "$wl" --no-e2e --no-cpu-baseline $extra > "$OUT/${wl}_h${h}.json" 2> "$OUT/${wl}_h${h}.err"
    python - "$OUT/${wl}_h${h}.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
m = d["roofline_merge"]
print(sys.argv[1], "%.3f G" % (d["value"] / 1e9), "ms/step %.4f" % d["ms_per_step"],
      "ingest us %.1f" % d["roofline"]["avg_launch_us"], "merge us %.1f" % m["avg_launch_us"],
      "sb", m["superbuckets"], "peak", m["peak_superbucket_entries"], "cap", m["superbucket_capacity"], flush=True)
PY
  done
done
