#!/bin/bash
# Landmark records gathered lazily (the one-launch evaluations no longer gather
# them; SKIP_PREP calls refresh them): full GPU suite, then the c2 step and
# rank 0's shard of an 8-way split with MVBA_EVAL_GATHER=1 (in-launch gather)
# against the default, alternated twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03k2}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_gpu_$TAG.log | head; exit $rc; }
summ() { python3 -c "
import json,sys
for ln in open('$1'):
    if ln.startswith('{'):
        d=json.loads(ln)
        print('  %s: step %.2f us  value %.4g' % ('$2', 1e3*d['ms_per_step'], d['value']))
"; }
for k in 1 2; do
  for n in 1 8; do
    for v in 1 0; do
      f=$OUT/gather_${n}_${v}_${k}_$TAG.log
      timeout -k 10 200 env MVBA_EVAL_GATHER=$v python3 bench.py --shard-of $n --steps 200 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 0 > $f 2>&1 || { tail -3 $f; exit 1; }
      summ $f "N=$n gather=$v"
    done
  done
done
exit 0
