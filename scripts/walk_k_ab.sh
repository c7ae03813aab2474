#!/bin/bash
# A/B of the bit-sliced walk's sets per lane (ULG_SLICED_K=small,layer6):
# single calls (score_probe) and the default bench line.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/walk_k
mkdir -p ${OUT}
for k in ${KS:-"2,4" "2,1" "1,1" "2,2" "2,8"}; do
  export ULG_SLICED_K=$k
  timeout -k 10 150 python -u scripts/score_probe.py --cases c3 c5 --reps 10 > ${OUT}/probe_${k/,/_}.log 2>&1
  timeout -k 10 150 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-search --no-c4 > ${OUT}/bench_${k/,/_}.json 2> ${OUT}/bench_${k/,/_}.err
  echo "K=$k $(grep -ho '"case": "c[35]".*"layers_ms": \[[0-9.]*' ${OUT}/probe_${k/,/_}.log | sed 's/"n".*"layers_ms"/ms/' | tr '\n' ' ') bench $(python3 -c "import json;d=json.load(open('${OUT}/bench_${k/,/_}.json'));print(round(d['ms_per_step'],4), round(d['value']/1e9,3), d.get('single_call_ms'))")"
done
