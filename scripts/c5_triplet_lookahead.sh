mkdir -p gpurun_out/c5t
for th in 1 8; do
  ULG_TRIPLET_THREADS=$th timeout -k 10 120 python scripts/c5_triplet.py --n 24 --N 20000 --extra 0.0 > gpurun_out/c5t/n24_t$th.json 2> gpurun_out/c5t/n24_t$th.err || exit $?
done
ULG_TRIPLET_THREADS=8 ULG_TRIPLET_TRACE=1 timeout -k 10 480 python scripts/c5_triplet.py --extra 0.0 > gpurun_out/c5t/n32_t8.json 2> gpurun_out/c5t/n32_t8.err
echo rc=$?
