# A/B of the exact replay's prefetch modes (ULG_EXACT_PF bit 0: decrease-key entries, bit 1: pop 5 levels ahead)
mkdir -p gpurun_out
for m in ${MODES:-0 1 2 3}; do
  ULG_EXACT_PF=$m timeout -k 10 200 python -u scripts/probe_exact.py c3 > gpurun_out/ab_pf$m.log 2>&1 || exit 1
done
