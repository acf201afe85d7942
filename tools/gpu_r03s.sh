#!/bin/bash
# c5 (depth blocks) and rank 0's shard of the 8-way c4 split on the current build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03s}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python3 bench.py --config c5 --steps 10 --no-cpu-baseline > $OUT/bench_c5_$TAG.log 2>&1 || { tail -5 $OUT/bench_c5_$TAG.log; exit 1; }
python3 tools/bench_summary.py $OUT/bench_c5_$TAG.log
timeout -k 10 500 python3 bench.py --config c4 --shard-of 8 --steps 5 --ba-iters 3 --no-cpu-baseline > $OUT/bench_c4_shard8_$TAG.log 2>&1 || { tail -5 $OUT/bench_c4_shard8_$TAG.log; exit 1; }
python3 tools/bench_summary.py $OUT/bench_c4_shard8_$TAG.log
exit 0
