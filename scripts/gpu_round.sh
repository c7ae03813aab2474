#!/bin/bash
# GPU-box runner: parity tests, then the bench, then (optionally) a rocprofv3
# kernel-trace of a short bench.  Every GPU step has its own time limit; a
# crash/abort/timeout (exit code other than 0/1 from pytest, non-zero from
# the rest) ends the script there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-run}
# heartbeat: long single tests print nothing until they finish
( while sleep 45; do date +%T >> gpurun_out/${TAG}_heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -n 30 gpurun_out/${TAG}_pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  rc=$?
  echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.json; tail -n 5 gpurun_out/${TAG}_bench.err
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ "${PROFILE:-0}" = "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err
  rc=$?
  echo "rocprof rc=$rc"; tail -n 5 gpurun_out/${TAG}_prof.err
  find gpurun_out/${TAG}_prof -name "*stats*" | head
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
exit 0
