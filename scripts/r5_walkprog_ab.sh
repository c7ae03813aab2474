#!/bin/bash
# A/B of the table-driven walk (walk_prog 1) against the unrolled recursion
# (walk_prog 0): lists (digests, C3 oracle), single-call times, per-wave walk
# clocks, sets-per-lane variants, then the scorer's GPU tests.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5wp}
mkdir -p $OUT
for wp in 1 0; do
  timeout -k 10 240 python3 scripts/score_probe.py --cases small c2 c3 c5 --reps 10 --options walk_prog=$wp > $OUT/probe_wp$wp.log 2>&1
  timeout -k 10 240 python3 scripts/score_probe.py --cases c3 c5 --reps 10 --options walk_prog=$wp,score_streams=1 > $OUT/probe1s_wp$wp.log 2>&1
  timeout -k 10 120 python3 scripts/walk_clock.py --case c3 --options walk_prog=$wp --out $OUT/wc$wp > $OUT/wclock_wp$wp.log 2>&1
done
for k in 2 8; do
  ULG_SLICED_K=$k timeout -k 10 240 python3 scripts/score_probe.py --cases c3 c5 --reps 10 --options walk_prog=1 > $OUT/probe_k$k.log 2>&1
done
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cbic.py tests/test_gpu_slots.py > $OUT/pytest.log 2>&1
echo all ok
