#!/bin/bash
# Pipelined CG batches (MVBA_CG_PIPE=1, default) against waiting on every batch
# (MVBA_CG_PIPE=0): solver tests, then bench lines (no profiler) at c2 (x3
# alternated) and c3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03j2}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_solver_gpu.py tests/test_solver_forms_gpu.py tests/test_deterministic_gpu.py tests/test_edge_cases.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?; tail -2 $OUT/pytest_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_$TAG.log | head; exit $rc; }
ba() { python3 -c "
import json
for ln in open('$1'):
    if ln.startswith('{'):
        d=json.loads(ln); b=d['ba']; bd=d.get('ba_deterministic',{})
        print('  %s: LM %.1f it/s, %d CG, %.2f us per CG iteration; det %.1f it/s, %d CG, %.2f us' % ('$2', b['iters_per_s'], b['cg_iterations'], 1e3*b['ms_per_cg_iteration'], bd.get('iters_per_s',0), bd.get('cg_iterations',0), 1e3*bd.get('ms_per_cg_iteration',0)))
"; }
for cfg in c2 c2 c2 c3; do
  for v in 0 1; do
    if [ $cfg = c3 ]; then A="--config c3 --steps 3 --ba-iters 3"; else A="--steps 5"; fi
    f=$OUT/pipe_${cfg}_${v}_$RANDOM.log
    timeout -k 10 400 env MVBA_CG_PIPE=$v python3 bench.py --no-cpu-baseline --mesh-subdiv 0 $A > $f 2>&1 || { tail -3 $f; exit 1; }
    ba $f "$cfg pipe=$v"
  done
done
exit 0
