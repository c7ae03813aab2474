#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes over the C3 bench, then the per-launch
# traffic summary of the roofline unit: layer 6 without variable 0 =
# score_layer_kernel<6, 1, V> + walk_sliced_kernel<6, 1, K>, per launch (one
# of the 3 stream groups: 2,557,324 / 3 sets on average).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-pmct}
bash scripts/pmc_round.sh FETCH_SIZE WRITE_SIZE || exit $?
F=$(find gpurun_out/${TAG:-pmc}/p1 gpurun_out/pmc/p1 -name "*counter_collection.csv" 2>/dev/null | head -1)
W=$(find gpurun_out/${TAG:-pmc}/p2 gpurun_out/pmc/p2 -name "*counter_collection.csv" 2>/dev/null | head -1)
python3 scripts/pmc_summarize.py "$F" "$W" "score_layer_kernel<6, 1,;walk_sliced_kernel<6, 1," c3 852441 \
    gpurun_out/pmc_traffic.json "score_layer_6_rest + walk_6_rest"
