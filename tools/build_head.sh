#!/bin/bash
# Build libsdp.so from the committed HEAD sources into build_ab/libsdp_head.so (A/B baseline).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C $ROOT archive HEAD spark-df-profiling_amd/csrc include | tar -x -C $T
cd $T/spark-df-profiling_amd/csrc
for f in *.hip *.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -mcode-object-version=5 \
     -x hip -c $f -o $T/$f.o &
done
wait
mkdir -p $ROOT/build_ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/build_ab/libsdp_head.so $T/*.o
rm -rf $T
echo built build_ab/libsdp_head.so from $(git -C $ROOT rev-parse --short HEAD)
