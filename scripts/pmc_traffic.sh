#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes over the C3 bench, then the per-launch
# traffic summary of the roofline unit: layer 6 without variable 0 =
# score_layer_kernel<6, 1, V> + walk_kernel<6, 1>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-pmct}
bash scripts/pmc_round.sh FETCH_SIZE WRITE_SIZE || exit $?
F=$(find gpurun_out/${TAG:-pmc}/p1 gpurun_out/pmc/p1 -name "*counter_collection.csv" 2>/dev/null | head -1)
W=$(find gpurun_out/${TAG:-pmc}/p2 gpurun_out/pmc/p2 -name "*counter_collection.csv" 2>/dev/null | head -1)
python3 scripts/pmc_summarize.py "$F" "$W" "score_layer_kernel<6, 1,;walk_kernel<6, 1>" c3 2557324 \
    gpurun_out/pmc_traffic.json "score_layer_6_rest + walk_6_rest"
