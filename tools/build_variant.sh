#!/bin/bash
# Build the C ABI with extra compiler flags into build_ab/libstereo_hip_<name>.so (A/B and diagnostic builds).
#   bash tools/build_variant.sh diag "-DWG_EXP=1024"
set -e
NAME=$1
FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$ROOT/build_ab/obj_$NAME
mkdir -p "$OBJ"
pids=()
for f in "$ROOT"/stereo_depth_estimation_amd/csrc/*.hip; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I"$ROOT/include" $FLAGS \
        -c "$f" -o "$OBJ/$(basename "$f" .hip).o" &
    pids+=($!)
done
for f in "$ROOT"/stereo_depth_estimation_amd/csrc/*.cpp; do
    g++ -O3 -std=c++17 -fPIC -Wall -pthread -I"$ROOT/include" -c "$f" -o "$OBJ/$(basename "$f" .cpp).cpp.o" &
    pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o "$ROOT/build_ab/libstereo_hip_$NAME.so" "$OBJ"/*.o -lz
rm -rf "$OBJ"
echo "build_ab/libstereo_hip_$NAME.so"
