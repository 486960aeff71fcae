set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r03 PMC_WLS="cfg2 cfg3 cfg4 cfg5" BENCH_WLS="cfg2 cfg3 cfg4 cfg5 cfg4_10m" bash tools/measure.sh
