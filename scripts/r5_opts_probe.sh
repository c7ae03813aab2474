#!/bin/bash
# Option A/B on the final tree: single calls (score_probe) per option set,
# alternating two rounds, then the share probe per option set.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5op}
mkdir -p $OUT
for rep in 1 2; do for o in ${OPTS_LIST:-score_small_layers=4 score_small_layers=3}; do
  timeout -k 10 200 python3 scripts/score_probe.py --cases c2 c3 c5 --reps 10 --options $o > $OUT/p_${o}_$rep.log 2>&1
  echo "$o rep=$rep $(grep -h '"case"' $OUT/p_${o}_$rep.log | sed -E 's/.*"case": "([a-z0-9]+)".*"digest": "([0-9a-f]+)".*"ms_median": ([0-9.]+).*/\1 \2 \3/' | tr '\n' ' ')"
done; done
for o in ${SHARE_OPTS:-walk_small_sets=0 score_small_layers=3}; do
  timeout -k 10 300 python3 scripts/share_probe.py --config c3 --options $o > $OUT/share_$o.log 2>&1
  echo "share $o: $(tail -1 $OUT/share_$o.log | cut -c1-330)"
done
