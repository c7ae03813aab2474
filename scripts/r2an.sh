# Round-2 r2an: batched presence gather A/B (ULG_PRES_NB / waves-per-EU builds) and the scorer's GPU tests
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in urlearning-cpp_amd/libulg.so abbuild/nb0/libulg.so abbuild/nb8/libulg.so abbuild/nb32/libulg.so abbuild/nb16w4/libulg.so abbuild/nb8w4/libulg.so; do
    ULG_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/score_time.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r2an_ab.log || exit 1
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_cbic.py tests/test_gpu_fullsize.py tests/test_gpu_c3_dag.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2an_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r2an_tests.log
exit $rc
