#!/bin/bash
# Round 3: wide-layer tests, C4 probe + bench, triplet tests, C5 sparse triplet.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c5t
TAG=${TAG:-r3}
( while sleep 45; do date +%T >> gpurun_out/${TAG}_heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_c45.py -x -v --timeout 380 --timeout-method thread > gpurun_out/${TAG}_wide_tests.log 2>&1 || { tail -20 gpurun_out/${TAG}_wide_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_wide_tests.log
timeout -k 10 100 python -u scripts/c4_probe.py 29 23 9 7 > gpurun_out/${TAG}_c4probe.log 2>&1 || exit 1
cat gpurun_out/${TAG}_c4probe.log
timeout -k 10 200 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-search > gpurun_out/${TAG}_c4_bench.json 2> gpurun_out/${TAG}_c4_bench.err || exit 1
python -c "import json;print('c4 ms_per_step', json.load(open('gpurun_out/${TAG}_c4_bench.json'))['ms_per_step'])"
[ "${TRIPLET:-1}" = "1" ] || exit 0
timeout -k 10 300 python -u -m pytest tests/test_gpu_triplet.py -x -v --timeout 250 --timeout-method thread > gpurun_out/${TAG}_triplet_tests.log 2>&1 || { tail -20 gpurun_out/${TAG}_triplet_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_triplet_tests.log
ULG_TRIPLET_TRACE=1 timeout -k 10 400 python -u scripts/c5_triplet.py --extra 0.0 > gpurun_out/c5t/${TAG}_n32.json 2> gpurun_out/c5t/${TAG}_n32_trace.log || { tail -5 gpurun_out/c5t/${TAG}_n32_trace.log; exit 1; }
cut -c1-600 gpurun_out/c5t/${TAG}_n32.json
