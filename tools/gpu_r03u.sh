#!/bin/bash
# k_eval_local with the landmark's offset / free flag loaded before K0:
# parity tests, then rank 0's shard of 8-, 4-, 2-way c2 splits against the
# previous build (tools/ab/head59b through MVBA_LIB), alternated twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03u}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_eval_forms_gpu.py tests/test_parity_gpu.py tests/test_full_size_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?; tail -2 $OUT/pytest_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_$TAG.log | head; exit $rc; }
summ() { python3 -c "
import json,sys
for ln in open('$1'):
    if ln.startswith('{'):
        d=json.loads(ln)
        print('  %s: step %.2f us' % ('$2', 1e3*d['ms_per_step']))
"; }
for k in 1 2; do
  for n in 8 4 2; do
    for v in base cur; do
      unset MVBA_LIB; [ $v = base ] && export MVBA_LIB=$PWD/tools/ab/head59b/libmvba.so
      f=$OUT/hoist_${n}_${v}_${k}_$TAG.log
      timeout -k 10 200 python3 bench.py --shard-of $n --steps 200 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 0 > $f 2>&1 || { tail -3 $f; exit 1; }
      summ $f "N=$n $v"
    done
  done
done
exit 0
