#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (each its own rocprofv3 --pmc run) over a
# short C3 bench WITH the search side, then the HBM traffic of one GPU
# order-graph sweep (all layer_pull*_kernel dispatches / sweeps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-pmcs}
mkdir -p gpurun_out/${TAG}
CMD="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
i=0
for ctrs in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc ${ctrs} --kernel-trace --output-format csv -d gpurun_out/${TAG}/p${i} -o run -- ${CMD} > gpurun_out/${TAG}/p${i}.log 2>&1
  rc=$?
  echo "pass $i ($ctrs) rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 gpurun_out/${TAG}/p${i}.log; exit $rc; fi
done
F=$(find gpurun_out/${TAG}/p1 -name "*counter_collection.csv" | head -1)
W=$(find gpurun_out/${TAG}/p2 -name "*counter_collection.csv" | head -1)
python3 scripts/pmc_search_summarize.py "$F" "$W" c3 25 gpurun_out/${TAG}/pmc_search_traffic.json
