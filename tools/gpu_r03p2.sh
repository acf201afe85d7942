#!/bin/bash
# c4 (8 sensors, 5M landmarks, 50M observations) whole on one GPU, final round-3 build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
f=$OUT/bench_c4_r03p2.log
timeout -k 10 900 python3 -u bench.py --config c4 --steps 5 --warmup 2 --ba-iters 2 --no-cpu-baseline > $f 2>&1 || { tail -5 $f; exit 1; }
python3 tools/bench_summary.py $f
exit 0
