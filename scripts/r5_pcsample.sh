#!/bin/bash
# PC sampling (rocprofv3, stochastic, cycles) of single C3 scoring calls on one
# stream: where the layer kernels' waves are when sampled, with stall reasons.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5pcs}
mkdir -p ${OUT}
timeout -k 10 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${METHOD:-stochastic} \
  --pc-sampling-unit ${UNIT:-cycles} --pc-sampling-interval ${INTERVAL:-65536} --output-format csv -d ${OUT}/pcs -o run \
  -- python3 scripts/score_probe.py --cases ${CASES:-c3} --reps 3 --options score_streams=1,score_graph=0 ${PROBE_ARGS:-} > ${OUT}/pcs.log 2>&1
echo "pc sampling ok"
ls -R ${OUT}/pcs | head -20
