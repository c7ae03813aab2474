# Round-2 r2ap: scorer floor without the presence gathers (timing probe, wrong lists) and C3 decision statistics
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in urlearning-cpp_amd/libulg.so abbuild/nopres/libulg.so; do
    echo "== $lib" | tee -a gpurun_out/r2ap_ab.log
    ULG_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/score_time.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r2ap_ab.log || exit 1
  done
done
timeout -k 10 120 python -u scripts/score_stats.py 2>&1 | grep -v amdgpu.ids > gpurun_out/r2ap_stats.log || exit 1
