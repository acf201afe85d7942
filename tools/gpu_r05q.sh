#!/bin/bash
# c4 same-box A/B: round-4 final library (tools/ab/r04x) vs the current tree,
# evaluation phase only, twice each alternating (the c4 headline moved from
# 7.36e9 (r04s box) to 6.49e9 (r05m box): code or box?)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r05q}
for k in 1 2; do
  for v in r04x cur; do
    if [ $v = cur ]; then unset MVBA_LIB; else export MVBA_LIB=$PWD/tools/ab/$v/libmvba.so; fi
    timeout -k 10 500 python bench.py --config c4 --steps 60 --warmup 3 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 0 > $OUT/c4eval_${v}_${k}_$TAG.log 2>&1 || { echo "bench failed ($v $k)"; exit 1; }
    echo "$v $k: $(python3 tools/bench_summary.py $OUT/c4eval_${v}_${k}_$TAG.log | tail -1 | cut -c1-160)"
  done
done
# c2 pass A with the pipelined loop gated to multi-segment chunks (tools/ab/pipe)
REPS="1" bash tools/gpu_kt_r05.sh $TAG "c2" "cur=MVBA_CG_GRAPH=1 pipe=MVBA_LIB=$PWD/tools/ab/pipe/libmvba.so" || exit 1
