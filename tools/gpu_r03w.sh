#!/bin/bash
# Second CG batch of 2 (default) against 4 (MVBA_CG_BATCH2=4): bench wall time
# per CG iteration at c2 and c3, alternating, no profiler.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
summ() { python3 -c "
import json
for ln in open('$1'):
    if ln.startswith('{'):
        d=json.loads(ln); b=d['ba']; t=d.get('ba_deterministic',{})
        print('  %-14s evals/s %.3g  CG %3d  %.1f us/CG it  %.1f LM it/s | det CG %s %.1f us/CG it' % ('$2', d['value'], b['cg_iterations'], 1e3*b['ms_per_cg_iteration'], b['iters_per_s'], t.get('cg_iterations'), 1e3*t.get('ms_per_cg_iteration', 0)))
"; }
for rep in 1 2; do
  for cfg in c2 c3; do
    for v in 2 4; do
      if [ $cfg = c3 ]; then A="--config c3 --steps 3 --ba-iters 5"; else A="--steps 20 --ba-iters 5"; fi
      f=$OUT/batch_${cfg}_${v}_$rep.log
      timeout -k 10 300 env MVBA_CG_BATCH2=$v python3 bench.py $A --no-cpu-baseline --mesh-subdiv 0 > $f 2>&1 || { tail -3 $f; exit 1; }
      summ $f "$cfg batch2=$v"
    done
  done
done
exit 0
