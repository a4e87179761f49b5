#!/bin/bash
# Builds a variant of librtamd.so with extra compile definitions, for A/B timing in one process:
#   tools/build_variant.sh NAME "-DKNOB=1 ..."  ->  realtimeraytracing_gradproject_amd/lib/variants/NAME/librtamd.so
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
DEFS="$*"
OUT=realtimeraytracing_gradproject_amd/lib/variants/$NAME
OBJ=build/variants/$NAME
mkdir -p "$OUT" "$OBJ"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -munsafe-fp-atomics $DEFS"
SRC=realtimeraytracing_gradproject_amd/csrc
/opt/rocm/bin/hipcc $FLAGS -c $SRC/rt_api.cpp -o $OBJ/rt_api.o &
/opt/rocm/bin/hipcc $FLAGS -c $SRC/rt_comm.cpp -o $OBJ/rt_comm.o &
/opt/rocm/bin/hipcc $FLAGS -c $SRC/rt_lbvh.hip -o $OBJ/rt_lbvh.o &
/opt/rocm/bin/hipcc $FLAGS -fno-slp-vectorize -mllvm -structurizecfg-skip-uniform-regions=1 -c $SRC/rt_trace.hip -o $OBJ/rt_trace.o &  # as the Makefile
/opt/rocm/bin/hipcc $FLAGS -c $SRC/rt_raster.hip -o $OBJ/rt_raster.o &
g++ -O2 -std=c++17 -fPIC -ffp-contract=off -c $SRC/rt_host.cpp -o $OBJ/rt_host.o &
wait
for o in rt_api rt_comm rt_lbvh rt_trace rt_raster rt_host; do [ -f $OBJ/$o.o ] || { echo "variant $NAME: $o failed"; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/librtamd.so $OBJ/*.o -ldl -Wl,-rpath,/opt/rocm/lib
echo "$OUT/librtamd.so"
