# Round-2 r2aj: exact-replay prefetch A/B (C3), triplet dense-replay A/B and its tests
set -u
mkdir -p gpurun_out
( while sleep 45; do date +%T >> gpurun_out/r2aj_heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for rep in 1 2; do
  for lib in urlearning-cpp_amd/libulg.so abbuild/wpe5/libulg.so abbuild/wpe6/libulg.so abbuild/wpe8/libulg.so; do
    ULG_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/score_time.py 2>&1 | tee -a gpurun_out/r2aj_wpe.log || exit 1
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_triplet.py -x -v --timeout 250 --timeout-method thread > gpurun_out/r2aj_triplet_tests.log 2>&1 || { tail -20 gpurun_out/r2aj_triplet_tests.log; exit 1; }
tail -3 gpurun_out/r2aj_triplet_tests.log
for d in 0 1; do
  ULG_TRIPLET_DENSE=$d ULG_TRIPLET_THREADS=16 timeout -k 10 200 python -u scripts/c5_triplet.py --n 24 --N 20000 --extra 0.0 > gpurun_out/r2aj_n24_dense$d.json 2> gpurun_out/r2aj_n24_dense$d.err || exit 1
  cut -c1-600 gpurun_out/r2aj_n24_dense$d.json
done
for m in ${MODES:-2 6 14 2 6 14}; do
  ULG_EXACT_PF=$m timeout -k 10 120 python -u scripts/probe_exact.py c3 2>&1 | sed "s/^/pf$m /" | tee -a gpurun_out/r2aj_ab_pf.log || exit 1
done
