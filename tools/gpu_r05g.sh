#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r05g}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -4 $OUT/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_kt_r05.sh $TAG "s8 c2" "cur=MVBA_CG_GRAPH=1 cs2=MVBA_CHUNK_SEGS=2 cs4=MVBA_CHUNK_SEGS=4 tiles=MVBA_POINT_W=tiles" || exit 1
bash tools/gpu_kt_r05.sh $TAG "c3" "cur=MVBA_CG_GRAPH=1 tiles=MVBA_POINT_W=tiles pa16=MVBA_PASS_A_SEGS=16" || exit 1
for cfg in s8 c2; do
  case $cfg in s8) A="--shard-of 8 --ba-iters 5";; c2) A="--ba-iters 5";; esac
  for m in 1 0; do
    MVBA_LM_MERGED=$m MVBA_CG_TIMING=1 timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline --mesh-subdiv 0 $A > $OUT/${cfg}_m${m}_$TAG.log 2>&1 || exit 1
    echo "$cfg merged=$m: $(python3 tools/bench_summary.py $OUT/${cfg}_m${m}_$TAG.log | tail -1 | sed 's/.*| LM/LM/')"
  done
done
