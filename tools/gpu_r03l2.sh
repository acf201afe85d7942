#!/bin/bash
# k_eval poll pacing: s_sleep 1 (in-tree) vs 4 vs 16 between a K1 wave's polls
# (tools/ab/sleepN through MVBA_LIB), c2 step and c3 step, alternated twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
summ() { python3 -c "
import json,sys
for ln in open('$1'):
    if ln.startswith('{'):
        d=json.loads(ln)
        print('  %s: step %.2f us' % ('$2', 1e3*d['ms_per_step']))
"; }
for k in 1 2; do
  for cfg in c2 c3; do
    for v in 1 4 16; do
      unset MVBA_LIB; [ $v != 1 ] && export MVBA_LIB=$PWD/tools/ab/sleep$v/libmvba.so
      if [ $cfg = c3 ]; then A="--config c3 --steps 20"; else A="--steps 200"; fi
      f=$OUT/poll_${cfg}_${v}_$k.log
      timeout -k 10 300 python3 bench.py $A --no-cpu-baseline --mesh-subdiv 0 --ba-iters 0 > $f 2>&1 || { tail -3 $f; exit 1; }
      summ $f "$cfg sleep=$v"
    done
  done
done
exit 0
