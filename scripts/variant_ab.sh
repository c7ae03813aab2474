#!/bin/bash
# Scorer variant A/B on one GPU: the cbic GPU tests, then per variant
# (VARIANTS) single calls at C3/C5/small (layers only) and the default bench
# line; the layer-stats build (ab/libulg_LAYER_STATS.so, if present) once per
# variant on C5 with one stream.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/variant_ab
mkdir -p ${OUT}
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_cbic.py -x -q --timeout 200 --timeout-method thread > ${OUT}/pytest.log 2>&1
  echo "tests: $(tail -1 ${OUT}/pytest.log)"
fi
for v in ${VARIANTS:-49 113}; do
  timeout -k 10 200 python -u scripts/score_probe.py --cases c3 c5 small --reps 10 --options score_variant=$v > ${OUT}/probe_$v.log 2>&1
  timeout -k 10 150 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-search --no-c4 --option score_variant=$v > ${OUT}/bench_$v.json 2> ${OUT}/bench_$v.err
  if [ -f ab/libulg_LAYER_STATS.so ]; then
    timeout -k 10 150 python -u scripts/score_probe.py --cases c5 --reps 1 --options score_variant=$v,score_streams=1 --lib ab/libulg_LAYER_STATS.so > ${OUT}/stats_$v.log 2>&1
  fi
  echo "variant $v: $(grep -ho '"case": "[a-z0-9]*", "n": [0-9]*.*"identical": [a-z]*.*"layers_ms": \[[0-9.]*' ${OUT}/probe_$v.log | sed 's/"N".*"identical"/identical/; s/"stored".*"layers_ms"/ms/' | tr '\n' ' ')"
  echo "   bench: $(python3 -c "import json;d=json.load(open('${OUT}/bench_$v.json'));print(round(d['ms_per_step'],4), round(d['value']/1e9,3), d.get('single_call_ms'), d.get('slot_check',{}).get('slots_lists_equal_oracle'))")"
done
