#!/bin/bash
# Rank 0's shard of an 8-way split of c5 (depth blocks, fp32 eval) and c3 on the final round-3 build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03h2}
OUT=gpurun_out
mkdir -p $OUT
for cfg in c5 c3; do
  f=$OUT/bench_${cfg}_shard8_$TAG.log
  timeout -k 10 400 python3 bench.py --config $cfg --shard-of 8 --steps 10 --ba-iters 3 --no-cpu-baseline > $f 2>&1 || { tail -5 $f; exit 1; }
  python3 tools/bench_summary.py $f
done
exit 0
