#!/bin/bash
# Build the bounds-checking test library (never shipped): build_ab/libsdp_dbg.so
set -e
cd "$(dirname "$0")/../spark-df-profiling_amd/csrc"
mkdir -p ../../build_ab/dbg
for f in sdp_abi.cpp sdp_numeric.hip sdp_hash.hip sdp_part.hip sdp_gram.hip sdp_bitmap.hip sdp_api.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -mcode-object-version=5 \
      -DSDP_DEBUG_BOUNDS -x hip -c $f -o ../../build_ab/dbg/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../build_ab/libsdp_dbg.so ../../build_ab/dbg/*.o
