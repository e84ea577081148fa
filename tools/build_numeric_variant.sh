#!/bin/bash
# Build build_ab/libsdp_NAME.so: sdp_numeric.hip compiled with extra -D flags,
# linked with the tree's other objects (spark-df-profiling_amd/csrc/build/).
# usage: tools/build_numeric_variant.sh NAME "-DP1_STAGES=4 ..."
set -e
cd "$(dirname "$0")/../spark-df-profiling_amd/csrc"
mkdir -p ../../build_ab/var_$1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -mcode-object-version=5 \
    $2 -x hip -c sdp_numeric.hip -o ../../build_ab/var_$1/sdp_numeric.hip.o
objs=$(ls build/*.o | grep -v sdp_numeric)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../build_ab/libsdp_$1.so $objs ../../build_ab/var_$1/sdp_numeric.hip.o
rm -rf ../../build_ab/var_$1
echo built build_ab/libsdp_$1.so
