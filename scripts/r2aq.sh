# Round-2 r2aq: C4 (all 30 variables, -p 29, MMPC) and C2 bench lines at HEAD
set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r2aq_c4_bench.json 2> gpurun_out/r2aq_c4_bench.err || { tail -5 gpurun_out/r2aq_c4_bench.err; exit 1; }
cat gpurun_out/r2aq_c4_bench.json
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r2aq_c2_bench.json 2> gpurun_out/r2aq_c2_bench.err || { tail -5 gpurun_out/r2aq_c2_bench.err; exit 1; }
cat gpurun_out/r2aq_c2_bench.json
