#!/bin/bash
# Build libsdp.so with one constant of sdp_part.hip changed, into build_ab/ (A/B runs via SDP_LIBRARY).
# Usage: tools/build_variant.sh NAME 'sed-expression'
set -e
NAME=$1; EXPR=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/spark-df-profiling_amd/csrc
T=$(mktemp -d)
mkdir -p $T/a/b && cp $C/*.hip $C/*.h $C/*.cpp $T/a/b/ && mkdir -p $T/include && cp $ROOT/include/sdp.h $T/include/ && T0=$T && T=$T/a/b
sed -i "$EXPR" $T/sdp_part.hip
for f in sdp_abi.cpp sdp_numeric.hip sdp_hash.hip sdp_part.hip sdp_gram.hip sdp_bitmap.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -mcode-object-version=5 \
     -I$C -x hip -c $T/$f -o $T/$f.o &
done
wait
mkdir -p $ROOT/build_ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/build_ab/libsdp_$NAME.so $T/*.o
rm -rf $T0
echo built build_ab/libsdp_$NAME.so
