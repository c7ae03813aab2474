# wide-walk checks: tests/test_gpu_wide.py, then C1 at lambda 0.5 timed and with walk statistics
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${TAG:-r2ab}
timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_wide.py > gpurun_out/${T}_wide.log 2>&1 && \
timeout -k 10 300 python -u scripts/c1_probe.py 0.5 --no-profile --digest gpurun_out/${T}_c1.json > gpurun_out/${T}_c1_time.log 2>&1 && \
ULG_WALK_STATS=1 timeout -k 10 300 python -u scripts/c1_probe.py 0.5 > gpurun_out/${T}_c1_stats.log 2>&1
