set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/ingest_probe
