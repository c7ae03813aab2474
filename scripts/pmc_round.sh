#!/bin/bash
# PMC passes for the roofline (separate --pmc runs, kernel-trace only; no
# sys/runtime traces).  FETCH_SIZE and WRITE_SIZE in their own passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-pmc}
mkdir -p gpurun_out/${TAG}
CMD="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-search ${BENCH_ARGS:-}"
timeout -k 10 120 rocprofv3 -L > gpurun_out/${TAG}/counters.txt 2>&1 || true
i=0
for ctrs in "${@}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc ${ctrs} --kernel-trace --output-format csv -d gpurun_out/${TAG}/p${i} -o run -- ${CMD} > gpurun_out/${TAG}/p${i}.log 2>&1
  rc=$?
  echo "pass $i ($ctrs) rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 gpurun_out/${TAG}/p${i}.log; exit $rc; fi
done
exit 0
