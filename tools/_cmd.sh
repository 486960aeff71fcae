set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for w in cfg2 cfg3; do
timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-e2e --no-kernel-events > gpurun_out/bench_${w}_noev.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_${w}_noev.json'));print('$w noev', round(d['value']/1e9,2), 'G ev/s', round(d['ms_per_step'],4))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$w -o run -- python3 bench.py --workload $w --no-cpu-baseline --no-e2e --no-kernel-events > gpurun_out/prof_$w.log 2>&1 || exit 1
done
