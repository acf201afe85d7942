#!/bin/bash
# K2 with 3 waves per frame-part block (tools/ab/flin3, MVBA_FLIN_WAVES=3)
# against the in-tree 2: bench linearize at c2 and c3, alternated twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
summ() { python3 -c "
import json,sys
for ln in open('$1'):
    if ln.startswith('{'):
        d=json.loads(ln); l=d['linearize']
        print('  %s: linearize %.2f us (camera side %.2f, point side %.2f)' % ('$2', 1e3*l['kernel_ms'], 1e3*l['camera_side_ms'], 1e3*l['point_side_ms']))
"; }
for k in 1 2; do
  for cfg in c2 c3; do
    for v in 2 3; do
      unset MVBA_LIB; [ $v = 3 ] && export MVBA_LIB=$PWD/tools/ab/flin3/libmvba.so
      if [ $cfg = c3 ]; then A="--config c3 --steps 10"; else A="--steps 50"; fi
      f=$OUT/flin_${cfg}_${v}_$k.log
      timeout -k 10 300 python3 bench.py $A --no-cpu-baseline --mesh-subdiv 0 --ba-iters 0 > $f 2>&1 || { tail -3 $f; exit 1; }
      summ $f "$cfg waves=$v"
    done
  done
done
exit 0
