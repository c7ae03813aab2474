# A/B of the wide-walk straggler budget (ULG_STRAG_BUDGET = log2 steps) on C1 lambda 0.5 and C4 per variable
mkdir -p gpurun_out
( while sleep 45; do date +%T >> gpurun_out/ab_heartbeat; done ) &
HB=$!
for b in ${BUDGETS:-13 11 9}; do
  ULG_STRAG_BUDGET=$b timeout -k 10 200 python -u scripts/c1_probe.py 0.5 --no-profile > gpurun_out/ab_b${b}_c1.log 2>&1 || { kill $HB; exit 1; }
  ULG_STRAG_BUDGET=$b timeout -k 10 300 python -u scripts/c4_probe.py > gpurun_out/ab_b${b}_c4.log 2>&1 || { kill $HB; exit 1; }
done
kill $HB
