#!/bin/bash
# The bench's timed loop with different steps in flight (--slots) and walk
# sets per lane (ULG_SLICED_K=small,layer6), alternating two rounds.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5slots}
mkdir -p $OUT
for rep in 1 2; do
  for sl in ${SLOTS:-3 4 6}; do
    for kk in ${KS:-2,4}; do
      ULG_SLICED_K=$kk timeout -k 10 200 python3 bench.py --steps 40 --warmup 6 --slots $sl --no-cpu-baseline --no-search --no-c4 > $OUT/s${sl}_k${kk}_${rep}.json 2> $OUT/s${sl}_k${kk}_${rep}.err
      echo "slots=$sl k=$kk rep=$rep $(python3 -c "import json;d=json.load(open('$OUT/s${sl}_k${kk}_${rep}.json'));print(round(d['value']/1e9,3), round(d['ms_per_step'],4))")"
    done
  done
done
