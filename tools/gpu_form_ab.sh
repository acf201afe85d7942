#!/bin/bash
# Evaluation launch form, MVBA_EVAL_MODE=fused|local, alternated twice, on whole
# configs (c2, c3 ...) and shard rehearsals (sN: rank 0's shard of an N-way
# split of c2). usage: tools/gpu_form_ab.sh TAG "c2 c3 s2 s4 s8"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/form_${1:-ab}
mkdir -p $OUT
for rep in 1 2; do
  for w in ${2:-s2 s4 s8}; do
    case $w in
      s*) a="--shard-of ${w#s} --steps 500";;
      c3) a="--config c3 --steps 30";;
      *) a="--config $w --steps 500";;
    esac
    for m in fused local; do
      MVBA_EVAL_MODE=$m timeout -k 10 300 python3 bench.py $a --ba-iters 0 --no-cpu-baseline \
        --mesh-subdiv 0 > $OUT/${w}_${m}_$rep.log 2>&1 || { echo "$w $m failed"; tail -5 $OUT/${w}_${m}_$rep.log; exit 1; }
      echo "$w $m $rep: $(python3 tools/bench_summary.py $OUT/${w}_${m}_$rep.log)"
    done
  done
done
