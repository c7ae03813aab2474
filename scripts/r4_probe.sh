#!/bin/bash
# Round-4 scorer probe on one GPU (each GPU step under its own time limit,
# chained so the first failure ends the call):
#  1. one call at a time (1 slot, 1 stream): bench line + rocprofv3 kernel
#     trace/stats of the same command (timeline and per-kernel averages);
#  2. SQ counter passes and the FETCH_SIZE / WRITE_SIZE passes over the same
#     command (separate --pmc runs, kernel trace only).
# TAG names the output directory under gpurun_out/; BENCH_ARGS adds options.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r4probe}
OUT=gpurun_out/${TAG}
mkdir -p ${OUT}
CMD="python3 bench.py --steps 10 --warmup 3 --slots 1 --option score_streams=1 --no-cpu-baseline --no-search --no-c4 ${BENCH_ARGS:-}"
timeout -k 10 180 ${CMD} > ${OUT}/bench.json 2> ${OUT}/bench.err
echo "bench: $(head -c 400 ${OUT}/bench.json)"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d ${OUT}/trace -o run -- ${CMD} > ${OUT}/trace.log 2>&1
echo "trace ok"
if [ "${PMC:-1}" = "1" ]; then
  i=0
  for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES" \
              "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
              "SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_TRANS_F64 SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT" \
              "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc ${ctrs} --kernel-trace --output-format csv -d ${OUT}/p${i} -o run -- ${CMD} > ${OUT}/p${i}.log 2>&1
    echo "pmc pass $i ok"
  done
fi
