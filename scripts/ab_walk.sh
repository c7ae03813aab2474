#!/bin/bash
# A/B of the walk forms on the GPU box: parity tests, then the C3 bench
# (scoring only) per ULG_SLICED_K setting.  Every GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abw
timeout -k 10 300 python -u -m pytest tests/test_gpu_cbic.py -m gpu -x -q --timeout 120 --timeout-method thread -k "walk_forms or variants" > gpurun_out/abw/pytest.log 2>&1 || { tail -30 gpurun_out/abw/pytest.log; exit 1; }
tail -2 gpurun_out/abw/pytest.log
# CASES: space-separated ULG_SLICED_K[:ULG_LANE_NW] settings
for c in ${CASES:-4 1 1:2}; do
  k=${c%%:*}; w=1; [ "$c" != "$k" ] && w=${c##*:}
  ULG_SLICED_K=$k ULG_LANE_NW=$w timeout -k 10 180 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-search > gpurun_out/abw/bench_${k}_${w}.json 2> gpurun_out/abw/bench_${k}_${w}.err || exit $?
  python -c "import json,sys;d=json.loads(open('gpurun_out/abw/bench_${k}_${w}.json').read().strip().splitlines()[-1]);print('K=$k NW=$w',round(d['ms_per_step'],4),'ms', {x:y for x,y in d['kernel_ms_one_step'].items() if 'walk' in x})"
done
