#!/bin/bash
# GPU box: the N = 2 multi-rank path rehearsed on ONE GPU (two gloo ranks share it), both watermark
# valves, CFG2 (one-phase) and CFG5 (two-phase).  Numbers are never reported: the exchange is host-staged.
set -o pipefail
mkdir -p gpurun_out
for w in cfg2 cfg5; do
  for v in device host; do
    timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
      bench.py --gpus 2 --dist-backend gloo --workload $w --steps 6 --warmup 2 --valve $v --no-cpu-baseline > gpurun_out/reh_${w}_$v.json 2> gpurun_out/reh_${w}_$v.err || { tail -20 gpurun_out/reh_${w}_$v.err; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/reh_${w}_$v.json').read().strip().splitlines()[-1]);print('$w $v', round(d['value']/1e9,3), 'G ev/s', 'ms/step', round(d['ms_per_step'],2), 'host_issue', round(d['host_issue_ms_per_step'],2), d['config']['exchange'])"
  done
done
