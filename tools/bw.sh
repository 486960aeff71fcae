#!/bin/bash
# Development: one short bench line per workload given (default cfg2..cfg5), no CPU / e2e legs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for w in ${@:-cfg2 cfg3 cfg4 cfg5}; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-e2e > gpurun_out/b.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$w', round(d['value']/1e9,2), 'G ev/s', round(d['ms_per_step'],4), {k: round(v*1e3,1) for k,v in d['device_ms_per_step'].items()}, 'host', round(d['host_issue_ms_per_step']*1e3,1), 'sb', d['config']['superbuckets'], 'frac', round(d['roofline']['frac'],3), round(d['roofline_merge']['frac'],3))"
done
