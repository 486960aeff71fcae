#!/bin/bash
# GPU box: one rank over RCCL through bench.py's N > 1 code path (--force-collectives): the packed
# exchange's all-to-all, the device valve's all-reduce and the per-rank load gather run in RCCL.
# Not a scaling measurement (the all-to-all is the rank's own segment).
set -o pipefail
mkdir -p gpurun_out
for w in cfg2 cfg5; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 \
    bench.py --gpus 1 --dist-backend nccl --force-collectives --workload $w --no-cpu-baseline > gpurun_out/rccl_n1_$w.json 2> gpurun_out/rccl_n1_$w.err || { tail -20 gpurun_out/rccl_n1_$w.err; exit 1; }
  python3 tools/summ.py "rccl n1" gpurun_out/rccl_n1_$w.json
done
