set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 180 --timeout-method thread -x -k "padded or golden" > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -15 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
WORLD_SIZE=2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 6 --warmup 2 --dist-backend gloo --workload cfg2 > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err || { tail -20 gpurun_out/bench_gloo2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_gloo2.json'));print(d['value']/1e9, d['config']['parallelism'], d['device_ms_per_step'])"
