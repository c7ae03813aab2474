# Round-2 r2ao: per-kernel times of the batched presence gather builds
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in urlearning-cpp_amd/libulg.so abbuild/nb0/libulg.so abbuild/nb8/libulg.so abbuild/nb32/libulg.so; do
    ULG_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/score_kernels.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r2ao_kernels.log || exit 1
  done
done
