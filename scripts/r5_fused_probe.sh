#!/bin/bash
# score_fused A/B: single-call timings and digests (score_probe) per setting,
# alternating two rounds, then one kernel trace per setting at C3.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5fu}
mkdir -p $OUT
for rep in 1 2; do for f in ${FS:-0 3 4}; do
  timeout -k 10 200 python3 scripts/score_probe.py --cases ${CASES:-small c2 c3 c5} --reps 10 --options score_fused=$f > $OUT/f${f}_$rep.log 2>&1
  echo "fused=$f rep=$rep $(grep -h '"case"' $OUT/f${f}_$rep.log | sed -E 's/.*"case": "([a-z0-9]+)".*"digest": "([0-9a-f]+)".*"ms_median": ([0-9.]+).*/\1 \2 \3/' | tr '\n' ' ')"
done; done
for f in ${FS:-0 3 4}; do
  LIBS=urlearning-cpp_amd/libulg.so CASES=c3 OPTS=score_streams=1,score_fused=$f TAG=${TAG:-r5fu}/k$f bash scripts/r5_kernel_ab.sh
done
