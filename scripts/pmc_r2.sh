#!/bin/bash
# Round-2 PMC passes (each its own rocprofv3 --pmc run, kernel-trace only):
#  1. scripts/bin/gather_probe -- known-byte streaming / gather kernels that
#     calibrate FETCH_SIZE and the raw TCC read-request counters on gfx950;
#  2. a short C3 bench with the search side -- the same counters over the
#     scorer's roofline pair and the GPU sweep, plus WRITE_SIZE and one SQ pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-pmc2}
mkdir -p gpurun_out/${TAG}
run() {  # name timeout counters... -- command
  local name=$1 tmo=$2; shift 2
  local ctrs=()
  while [ "$1" != "--" ]; do ctrs+=("$1"); shift; done
  shift
  timeout -k 10 ${tmo} rocprofv3 --pmc "${ctrs[@]}" --kernel-trace --output-format csv -d gpurun_out/${TAG}/${name} -o run -- "$@" > gpurun_out/${TAG}/${name}.log 2>&1
  local rc=$?
  echo "pass ${name} (${ctrs[*]}) rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 gpurun_out/${TAG}/${name}.log; exit $rc; fi
}
PROBE=./scripts/bin/gather_probe
run g_fetch 90 FETCH_SIZE -- ${PROBE}
run g_req 90 TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum -- ${PROBE}
run g_dram 90 TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_32B_sum -- ${PROBE}
BENCH="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
run b_fetch 240 FETCH_SIZE -- ${BENCH}
run b_write 240 WRITE_SIZE -- ${BENCH}
run b_req 240 TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum -- ${BENCH}
run b_dram 240 TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_32B_sum -- ${BENCH}
run b_sq 240 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES -- ${BENCH}
exit 0
