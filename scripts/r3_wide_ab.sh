#!/bin/bash
# Round 3: wide-layer host-walk options on C4 (whole step) and C1 (lambda
# 0.5), then the PMC traffic passes of the C3 scorer.  Each GPU step under its
# own limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r3k}
timeout -k 10 300 python -u scripts/c4_opts_ab.py "wide_host=4096,wide_host_threads=8,wide_host_first=0" \
    "wide_host=1024,wide_host_threads=16,wide_host_first=0" "wide_host=1024,wide_host_threads=16,wide_host_first=64" \
    "wide_host=1024,wide_host_threads=16,wide_host_first=512" "wide_host=4096,wide_host_threads=16,wide_host_first=64" \
    > gpurun_out/${TAG}_c4_ab.log 2>&1 || { tail -5 gpurun_out/${TAG}_c4_ab.log; exit 1; }
cat gpurun_out/${TAG}_c4_ab.log
[ "${C1:-1}" = "1" ] && { timeout -k 10 900 python -u scripts/c4_opts_ab.py --c1 \
    "score_variant=113,wide_pool=1,wide_host=4096,wide_host_threads=8,wide_host_first=0" \
    "score_variant=49,wide_pool=1,wide_host=4096,wide_host_threads=8,wide_host_first=0" \
    "score_variant=113,wide_pool=0,wide_host=4096,wide_host_threads=8,wide_host_first=0" \
    "score_variant=113,wide_pool=1,wide_host=0,wide_host_threads=8,wide_host_first=0" \
    "score_variant=113,wide_pool=1,wide_host=4096,wide_host_threads=8,wide_host_first=64" \
    > gpurun_out/${TAG}_c1_ab.log 2>&1 || { tail -5 gpurun_out/${TAG}_c1_ab.log; exit 1; }; cat gpurun_out/${TAG}_c1_ab.log; }
[ "${PMC:-1}" = "1" ] && { TAG=pmc3 bash scripts/pmc_traffic.sh > gpurun_out/${TAG}_pmc.log 2>&1 || { tail -5 gpurun_out/${TAG}_pmc.log; exit 1; }; tail -2 gpurun_out/${TAG}_pmc.log; }
exit 0
