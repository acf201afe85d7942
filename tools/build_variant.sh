#!/bin/bash
# Build another libmvba.so with extra compile definitions for a same-box A/B
# (tools/gpu_session.sh's ab step loads it through MVBA_LIB): tools/build_variant.sh NAME "-DX=1 ..."
set -eu
cd "$(dirname "$0")/.."
NAME=$1; shift
DEFS="$*"
OUT=tools/ab/$NAME
mkdir -p $OUT
SRCS=$(python3 -c "from multiview_amd.build import SOURCES; print(' '.join(SOURCES))")
pids=()
for s in $SRCS; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fopenmp -Wall -Wno-unused-function $DEFS \
    -x hip -c multiview_amd/csrc/$s -o $OUT/${s%.*}.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fopenmp -o $OUT/libmvba.so $OUT/*.o -L/opt/rocm/lib -lrccl
rm -f $OUT/*.o
echo $OUT/libmvba.so
