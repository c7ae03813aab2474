#!/bin/bash
# Builds an A/B copy of libulg.so with extra preprocessor definitions for
# cbic.hip only (the other objects come from urlearning-cpp_amd/build/):
#   scripts/build_variant.sh NAME "-DFOO=1 -DBAR"  -> urlearning-cpp_amd/ablib/NAME/libulg_NAME.so (travels to the GPU box; *.o and *.so stay out of git)
set -eu
cd "$(dirname "$0")/.."
NAME=$1; DEFS=${2:-}
OUT=urlearning-cpp_amd/ablib/$NAME
mkdir -p $OUT
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Xarch_host -mpopcnt -Xarch_host -mbmi2 -Wall -Wno-unused-function -Wno-unused-result"
/opt/rocm/bin/hipcc $FLAGS $DEFS -c -o $OUT/cbic.o urlearning-cpp_amd/csrc/cbic.hip
OBJS=$(ls urlearning-cpp_amd/build/*.o | grep -v -e '/cbic.o$' -e 'cbic_ru.o$')
/opt/rocm/bin/hipcc $FLAGS -shared -o $OUT/libulg_$NAME.so $OUT/cbic.o $OBJS
echo $OUT/libulg_$NAME.so
