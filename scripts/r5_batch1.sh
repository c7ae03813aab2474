#!/bin/bash
# Round-5 batch: C4 host-handover A/B, a single C3 call's kernel timeline
# (3 stream groups), and bench loop shapes (slots x streams).
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5b1
mkdir -p $OUT
timeout -k 10 600 python3 scripts/c4_opts_ab.py "" "wide_host_q=14" "wide_host_q=15" "wide_host_q=16" > $OUT/c4ab.log 2>&1
echo c4 ok
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/tl -o run -- python3 scripts/score_probe.py --cases c3 --reps 3 > $OUT/tl.log 2>&1
echo trace ok
for cfg in "3 1" "2 2" "3 2" "2 3"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --steps 40 --warmup 6 --slots $1 --option score_streams=$2 --no-cpu-baseline --no-search --no-c4 > $OUT/b_s$1_g$2.json 2> $OUT/b_s$1_g$2.err
  echo "slots=$1 streams=$2 $(python3 -c "import json;d=json.load(open('$OUT/b_s$1_g$2.json'));print(round(d['value']/1e9,3), round(d['ms_per_step'],4))")"
done
timeout -k 10 300 python3 scripts/gather_stats.py --lib urlearning-cpp_amd/diag/libulg_stats.so --cases c3 c5 > $OUT/gstats.jsonl 2> $OUT/gstats.err
echo gstats ok
