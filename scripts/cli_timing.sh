#!/bin/bash
# End-to-end command-line timing at C2/C3 (GPU box): CSV -> score -> .pss -> astar / triplet_astar.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cli
OUT=gpurun_out/cli
python - <<'PY'
import sys
sys.path.insert(0, "urlearning-cpp_amd")
import synth
for name, n, N in (("c2", 20, 10000), ("c3", 25, 10000)):
    X, _ = synth.gaussian_sem(n, N, 9200)
    synth.write_csv(f"/tmp/{name}.csv", X)
PY
B=urlearning-cpp_amd/bin
for c in c2:${CK2:-4} c3:${CK3:-6}; do
  name=${c%%:*}; k=${c##*:}
  t0=$(date +%s.%N)
  timeout -k 10 300 $B/score /tmp/$name.csv /tmp/$name.pss -f cBIC --lambda 2 -p $k > $OUT/${name}_score.log 2>&1 || exit $?
  t1=$(date +%s.%N)
  ls -la /tmp/$name.pss >> $OUT/${name}_score.log
  timeout -k 10 300 $B/astar /tmp/$name.pss -n /tmp/${name}_net --mode ${MODE:-exact} > $OUT/${name}_astar.log 2>&1 || exit $?
  t2=$(date +%s.%N)
  python3 -c "print('$name wall: score %.3f s, astar %.3f s' % ($t1 - $t0, $t2 - $t1))"
  cat $OUT/${name}_score.log $OUT/${name}_astar.log
done
