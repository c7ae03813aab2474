#!/bin/bash
# Round 3: exact replay with/without the speculative descent (C3, then two
# C5-sparse triplet clusters alone), and the C4 v=23 wide-walk breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r3w}
( while sleep 45; do date +%T >> gpurun_out/${TAG}_heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
ULG_WALK_STATS=1 timeout -k 10 100 python -u scripts/c4_probe.py 29 23 > gpurun_out/${TAG}_c4_v23_stats.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/ab_exact_spec.py --config c3 --modes 6 22 --fast 12 6 --reps 3 > gpurun_out/${TAG}_exact_ab.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_exact_ab.log
timeout -k 10 400 python -u scripts/ab_triplet_cluster.py --reps 1 > gpurun_out/${TAG}_triplet_ab.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_triplet_ab.log
