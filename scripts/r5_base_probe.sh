set -eu
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=r5base PMC=1 bash scripts/r4_probe.sh
TAG=r5base_mem CMD_ARGS="--cases c3 --options score_streams=1" bash scripts/pmc_mem.sh
