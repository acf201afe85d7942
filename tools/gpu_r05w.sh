#!/bin/bash
# c4 evaluation forms, same box: k_eval_local (default), split (prep + K1),
# fused (K0 blocks hand records to the K1 waves), twice each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r05w}
for k in 1 2; do
  for m in local split fused; do
    MVBA_EVAL_MODE=$m timeout -k 10 400 python bench.py --config c4 --steps 40 --warmup 3 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 0 > $OUT/c4form_${m}_${k}_$TAG.log 2>&1 || { echo "bench failed ($m $k)"; exit 1; }
    echo "$m $k: $(python3 tools/bench_summary.py $OUT/c4form_${m}_${k}_$TAG.log | tail -1 | cut -c1-170)"
  done
done
