#!/bin/bash
# Single-call timings (score_probe) per walk sets-per-lane setting
# (ULG_SLICED_K=layers<=5,layer6), alternating two rounds.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5k}
mkdir -p $OUT
for rep in 1 2; do for kk in ${KS:-2,4 2,8 4,8}; do
ULG_SLICED_K=$kk timeout -k 10 200 python3 scripts/score_probe.py --cases ${CASES:-c2 c3 c5} --reps 10 > $OUT/k${kk}_$rep.log 2>&1
echo "k=$kk rep=$rep $(grep -h '"case": "c[35]"' $OUT/k${kk}_$rep.log | sed -E 's/.*"case": "(c[0-9])".*"digest": "([0-9a-f]+)".*"ms_median": ([0-9.]+).*/\1 \2 \3/' | tr '\n' ' ')"
done; done
