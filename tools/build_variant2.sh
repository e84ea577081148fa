#!/bin/bash
# Build libsdp.so with extra compile flags and/or a sed edit of one source, into build_ab/ (A/B runs via SDP_LIBRARY).
# Usage: tools/build_variant2.sh NAME 'EXTRA_FLAGS' [FILE 'sed-expression']
set -e
NAME=$1; FLAGS=$2; FILE=$3; EXPR=$4
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/spark-df-profiling_amd/csrc
T0=$(mktemp -d); T=$T0/a/b
mkdir -p $T && cp $C/*.hip $C/*.h $C/*.cpp $T/ && mkdir -p $T0/include && cp $ROOT/include/sdp.h $T0/include/
if [ -n "$FILE" ]; then sed -i "$EXPR" $T/$FILE; fi
for f in $(cd $T && ls *.hip *.cpp); do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -mcode-object-version=5 \
     $FLAGS -x hip -c $T/$f -o $T/$f.o &
done
wait
mkdir -p $ROOT/build_ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/build_ab/libsdp_$NAME.so $T/*.o
rm -rf $T0
echo built build_ab/libsdp_$NAME.so
