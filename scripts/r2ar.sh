# Round-2 r2ar: lazy heap positions (DenseHeap::lazy) -- exact replay A/B at C3 (ULG_EXACT_LAZY 1 / 0, profiled once),
# then the search, DAG and triplet GPU tests with the default (lazy) replay
set -u
mkdir -p gpurun_out
( while sleep 45; do date +%T >> gpurun_out/r2ar_heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for z in 1 0 1 0; do
  ULG_EXACT_LAZY=$z timeout -k 10 150 python -u scripts/probe_exact.py c3 2>&1 | grep -v amdgpu.ids | sed "s/^/lazy$z /" | tee -a gpurun_out/r2ar_ab.log || exit 1
done
ULG_EXACT_PROF=1 timeout -k 10 150 python -u scripts/probe_exact.py c3 2>&1 | grep exact_prof | head -3 > gpurun_out/r2ar_prof.log || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_search_dag.py tests/test_gpu_c3_dag.py tests/test_gpu_triplet.py tests/test_gpu_timeout.py tests/test_gpu_scoped.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r2ar_tests.log 2>&1 || { tail -30 gpurun_out/r2ar_tests.log; exit 1; }
tail -3 gpurun_out/r2ar_tests.log
