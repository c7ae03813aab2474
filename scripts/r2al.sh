# Round-2 r2al: triplet tests, then C5 sparse (n=32) with the dense cluster replay
set -u
mkdir -p gpurun_out/c5t
( while sleep 45; do date +%T >> gpurun_out/r2al_heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -m pytest tests/test_gpu_triplet.py -x -v --timeout 250 --timeout-method thread > gpurun_out/r2al_triplet_tests.log 2>&1 || { tail -20 gpurun_out/r2al_triplet_tests.log; exit 1; }
tail -2 gpurun_out/r2al_triplet_tests.log
ULG_TRIPLET_THREADS=16 ULG_TRIPLET_TRACE=1 timeout -k 10 560 python -u scripts/c5_triplet.py --extra 0.0 > gpurun_out/c5t/r2al_n32_t16.json 2> gpurun_out/c5t/r2al_n32_t16_trace.log || { tail -5 gpurun_out/c5t/r2al_n32_t16_trace.log; exit 1; }
cut -c1-800 gpurun_out/c5t/r2al_n32_t16.json
