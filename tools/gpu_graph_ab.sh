#!/bin/bash
# same-box A/B of the CG loop: eager launches vs replayed hipGraph runs of
# MVBA_CG_GRAPH_RUN iterations (s8 = rank 0's 1/8 shard of c2, and c2), with the
# host-side split of the linear-solver time (MVBA_CG_TIMING=1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-gab}
for k in 1 2; do
for cfg in s8 c2; do
  case $cfg in s8) A="--shard-of 8 --ba-iters 5";; c2) A="--ba-iters 5";; esac
  for v in g0 g2 g10; do
    case $v in g0) E="MVBA_CG_GRAPH=0";; g2) E="MVBA_CG_GRAPH=1 MVBA_CG_GRAPH_RUN=2";; g10) E="MVBA_CG_GRAPH=1 MVBA_CG_GRAPH_RUN=10";; esac
    env $E MVBA_CG_TIMING=1 timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline --mesh-subdiv 0 $A > $OUT/${cfg}_${v}_${k}_$TAG.log 2>&1 || exit 1
    echo "$cfg $v $k: $(grep 'cg timing' $OUT/${cfg}_${v}_${k}_$TAG.log | tail -1 | sed 's/.*batches) | //')"
    python3 tools/bench_summary.py $OUT/${cfg}_${v}_${k}_$TAG.log | tail -1 | sed 's/.*| LM/LM/'
  done
done
done
