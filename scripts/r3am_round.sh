#!/bin/bash
# Round 3: the bench at its new defaults (3 steps in flight, one stream per
# context), its PMC traffic passes and kernel stats, and a 2-rank gloo
# rehearsal of the slotted exchange.  Each GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r3am}
( while sleep 45; do date +%T >> gpurun_out/${TAG}_heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['step_level']['frac'])"
TAG=${TAG}_pmc bash scripts/pmc_round.sh FETCH_SIZE WRITE_SIZE || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err || { tail -5 gpurun_out/${TAG}_prof.err; exit 1; }
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --device 0 --steps 6 --warmup 3 > gpurun_out/${TAG}_gloo2.json 2> gpurun_out/${TAG}_gloo2.err || { tail -5 gpurun_out/${TAG}_gloo2.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_gloo2.json'));print('gloo2', d['value'], d['ms_per_step'], d['astar']['ranks_agree'])"
