#!/bin/bash
# Memory-pipeline counters of the scorer (one PMC pass per group, kernel trace
# only): L1 accesses / L1->L2 requests and their latency, TA busy, L1 TLB
# (UTCL1) hits / misses / stalls, L2 hits / misses.  CMD_ARGS picks the probe.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc_mem}
mkdir -p ${OUT}
CMD="python3 scripts/score_probe.py --reps 2 ${CMD_ARGS:---cases c5 --options score_streams=1}"
i=0
for ctrs in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE" \
            "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_THRASHING_STALL_sum" \
            "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" \
            "TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_REQUEST_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc ${ctrs} --kernel-trace --output-format csv -d ${OUT}/p${i} -o run -- ${CMD} > ${OUT}/p${i}.log 2>&1
  echo "pmc pass $i ok"
done
