#!/bin/bash
# Single-call timings per score_streams setting (alternating two rounds),
# the strong-scaling share probe, then the default bench line.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5st}
mkdir -p $OUT
for rep in 1 2; do for s in ${SS:-2 3 4}; do
  timeout -k 10 200 python3 scripts/score_probe.py --cases c3 c5 --reps 10 --options score_streams=$s > $OUT/s${s}_$rep.log 2>&1
  echo "streams=$s rep=$rep $(grep -h '"case"' $OUT/s${s}_$rep.log | sed -E 's/.*"case": "([a-z0-9]+)".*"digest": "([0-9a-f]+)".*"ms_median": ([0-9.]+).*/\1 \2 \3/' | tr '\n' ' ')"
done; done
timeout -k 10 300 python3 scripts/share_probe.py --config c3 > $OUT/share_c3.log 2>&1
tail -1 $OUT/share_c3.log | cut -c1-400
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
head -c 600 $OUT/bench.json
