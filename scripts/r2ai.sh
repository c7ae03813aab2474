# search checks after a sweep-table change: the search test files, then the C3 bench's search metrics
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r2ai}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_search.py tests/test_gpu_search_dag.py tests/test_gpu_shard.py tests/test_gpu_c3_dag.py > gpurun_out/${T}_search.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
