set -o pipefail
cd $GRAFT_REPO_ROOT
for w in cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 120 python tools/ablate.py merge $w 128,136,192 >> gpurun_out/ablate_merge3.log 2>&1 || exit 1
done
cat gpurun_out/ablate_merge3.log
