#!/bin/bash
# Round-5 profile of the shipped scorer, on the bench's own command:
#  1. the default bench line (bench.json);
#  2. rocprofv3 --kernel-trace --stats of the same command;
#  3. PMC passes (one counter group per run, kernel trace only) of the timed
#     configuration without the search / C4 / CPU legs: FETCH_SIZE,
#     WRITE_SIZE, the TA / TCP memory-pipeline group, two SQ groups;
#  4. scripts/pmc_r5_summarize.py -> ${OUT}/pmc_scorer.json.
# Every GPU step runs under its own time limit; the first failure ends it.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5probe}
mkdir -p ${OUT}
FULL="python3 bench.py ${BENCH_ARGS:-}"
SHORT="python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-search --no-c4 ${BENCH_ARGS:-}"
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 400 ${FULL} > ${OUT}/bench.json 2> ${OUT}/bench.err
  echo "bench: $(head -c 300 ${OUT}/bench.json)"
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d ${OUT}/trace -o run -- ${FULL} > ${OUT}/trace.log 2>&1
  echo "trace ok"
fi
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" \
            "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE" \
            "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES" \
            "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc ${ctrs} --kernel-trace --output-format csv -d ${OUT}/p${i} -o run -- ${SHORT} > ${OUT}/p${i}.log 2>&1
  echo "pmc pass $i ok"
done
python3 scripts/pmc_r5_summarize.py ${OUT} > ${OUT}/pmc_scorer.json
echo "summary ok"
