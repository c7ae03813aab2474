set -eu
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r5k
for rep in 1 2; do for kk in 2,4 2,8 4,8; do
ULG_SLICED_K=$kk timeout -k 10 200 python3 scripts/score_probe.py --cases c2 c3 c5 --reps 10 > gpurun_out/r5k/k${kk}_$rep.log 2>&1
done; done
