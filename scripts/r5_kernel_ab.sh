#!/bin/bash
# Per-kernel durations of several libulg.so builds (LIBS): rocprofv3 kernel
# trace of single calls on one stream (CASES), one run per build.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5kab}
mkdir -p $OUT
for lib in ${LIBS}; do
  nm=$(basename $lib .so)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$nm -o run -- \
    python3 scripts/score_probe.py --lib $lib --cases ${CASES:-c3 c5} --reps 5 --options ${OPTS:-score_streams=1} > $OUT/$nm.log 2>&1 \
    || [ $? -eq 1 ]  # 1: lists differ (the timing-only probe builds); anything else ends the run
  echo "$nm ok"
done
