#!/bin/bash
# BASELINE config C5 on one GPU: n=32, N=50k, full skeleton, k=6 (SURVEY N9:
# with k unbounded the reference would score 2^31 sets per variable):
# CSV -> score -> .pss -> triplet_astar MEC (every triplet cluster has 32 > 26
# variables, so every A* is skipped and the MEC is empty), plus calc_dag_score.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c5
mkdir -p $OUT
python3 - <<'PY'
import sys
sys.path.insert(0, "urlearning-cpp_amd")
import synth
X, W = synth.gaussian_sem(32, 50000, 9700)
synth.write_csv("/tmp/c5.csv", X)
with open("/tmp/c5_full.csv", "w") as f:
    for i in range(32):
        f.write(",".join(["1"] * 32) + "\n")
PY
B=urlearning-cpp_amd/bin
timeout -k 10 600 $B/score /tmp/c5.csv /tmp/c5.pss -f cBIC --lambda 2 -p 6 -k /tmp/c5_full.csv > $OUT/score.log 2>&1 || { cat $OUT/score.log; exit 1; }
cat $OUT/score.log; ls -la /tmp/c5.pss
timeout -k 10 600 $B/triplet_astar /tmp/c5.pss -k /tmp/c5_full.csv -n /tmp/c5_mec > $OUT/triplet.log 2>&1 || { cat $OUT/triplet.log; exit 1; }
cat $OUT/triplet.log; cp /tmp/c5_mec.csv $OUT/; head -3 /tmp/c5_mec.csv
