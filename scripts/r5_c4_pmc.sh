#!/bin/bash
# Counters of the C4 wide-layer LDS replay (walk_wide_lds_kernel): SQ passes
# over C4 variable 23 (m = 17, the step's longest chain) with ULG_WALK_STATS
# printing every replay launch's iteration count, so instructions and wait
# cycles per replay iteration can be formed (scripts/c4_replay_summary.py).
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5c4pmc}
mkdir -p ${OUT}
CMD="python3 scripts/c4_probe.py 29 ${VARS:-23}"
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD" \
            "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  ULG_WALK_STATS=1 timeout -s KILL 150 rocprofv3 --pmc ${ctrs} --kernel-trace --output-format csv -d ${OUT}/p${i} -o run -- ${CMD} > ${OUT}/p${i}.log 2>&1
  echo "pmc pass $i ok"
done
