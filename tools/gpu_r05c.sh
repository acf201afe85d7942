#!/bin/bash
# round-5 iteration: full GPU suite, then the s8 / c2 bench with the CG timing split
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r05c}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -5 $OUT/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cfg in s8 c2; do
  case $cfg in s8) A="--shard-of 8 --ba-iters 3";; c2) A="--ba-iters 5";; esac
  for g in 1 0; do
    MVBA_CG_GRAPH=$g MVBA_CG_TIMING=1 timeout -k 10 300 python bench.py --steps 200 --no-cpu-baseline --mesh-subdiv 0 $A > $OUT/${cfg}_g${g}_$TAG.log 2>&1 || exit 1
    echo "$cfg graph=$g: $(grep 'cg timing' $OUT/${cfg}_g${g}_$TAG.log | tail -1)"
    python3 tools/bench_summary.py $OUT/${cfg}_g${g}_$TAG.log | tail -1
  done
done
