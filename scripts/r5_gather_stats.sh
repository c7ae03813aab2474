set -eu
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5gs
timeout -k 10 300 python3 scripts/gather_stats.py --lib urlearning-cpp_amd/diag/libulg_stats.so --cases c3 c5 > gpurun_out/r5gs/stats.jsonl 2> gpurun_out/r5gs/stats.err
cat gpurun_out/r5gs/stats.jsonl
