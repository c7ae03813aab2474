#!/bin/bash
# Per-kernel A/B of libulg builds: for each library (LIBS, default the
# in-tree one and ab/*.so) a C3+C5 single-call probe (layers only, one stream)
# under rocprofv3 --kernel-trace --stats.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/abk
mkdir -p ${OUT}
for lib in ${LIBS:-urlearning-cpp_amd/libulg.so ab/*.so}; do
  tag=$(basename ${lib} .so)
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d ${OUT}/${tag} -o run -- \
    python3 scripts/score_probe.py --cases ${CASES:-c3 c5} --reps 10 --options score_streams=1 --lib ${lib} \
    > ${OUT}/${tag}.log 2>&1
  echo "${tag}: $(grep -ho '"case": "c[35]".*"layers_ms": \[[0-9.]*' ${OUT}/${tag}.log | sed 's/"n".*"layers_ms"/ms/' | tr '\n' ' ')"
done
