#!/bin/bash
# Full GPU suite on the current build (frame-order back-substitution, size-based
# c_o order); evaluation modes at N = 1 and 2 (fused vs local); then bench
# lines (no profiler) of the previous build (tools/ab/base, MVBA_LIB) against
# the current one at c2 (alternated twice) and c3, plus the current build with
# the point-order back-substitution at c3 (MVBA_BACKSUB=point). The current
# build also inverts wide preconditioner blocks by Gauss-Jordan in LDS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03p}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_gpu_$TAG.log | head; exit $rc; }
summ() { python3 -c "
import json,sys
for ln in open('$1'):
    if ln.startswith('{'):
        d=json.loads(ln); r=d['roofline']
        print('  %s: step %.2f us  host enqueue %.2f us  K1 %.2f us  prep %.2f us' % ('$2', 1e3*d['ms_per_step'], 1e3*d['host_issue_ms_per_step'], 1e3*r['kernel_ms'], 1e3*r['prep_ms']))
"; }
for k in 1 2; do
  for n in 1 2; do
    for v in fused local; do
      f=$OUT/evm_${n}_${v}_${k}_$TAG.log
      timeout -k 10 200 env MVBA_EVAL_MODE=$v python3 bench.py --shard-of $n --steps 100 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 0 > $f 2>&1 || { tail -3 $f; exit 1; }
      summ $f "N=$n $v"
    done
  done
done
ba() { python3 -c "
import json
for ln in open('$1'):
    if ln.startswith('{'):
        d=json.loads(ln); b=d['ba']; bd=d.get('ba_deterministic',{})
        print('  %s: LM %.1f it/s, %d CG, %.2f us per CG iteration (linear solver %.2f ms); det %d CG %.2f us; eval step %.2f us' % ('$2', b['iters_per_s'], b['cg_iterations'], 1e3*b['ms_per_cg_iteration'], 1e3*b['linear_solver_s'], bd.get('cg_iterations',0), 1e3*bd.get('ms_per_cg_iteration',0), 1e3*d['ms_per_step']))
"; }
for cfg in c2 c2 c3; do
  for v in base cur bsp; do
    unset MVBA_LIB MVBA_BACKSUB
    [ $v = base ] && export MVBA_LIB=$PWD/tools/ab/base/libmvba.so
    [ $v = bsp ] && export MVBA_BACKSUB=point
    if [ $cfg = c3 ]; then A="--config c3 --steps 3 --ba-iters 3"; else A="--steps 10"; fi
    f=$OUT/ba_${cfg}_${v}_$RANDOM.log
    timeout -k 10 400 python3 bench.py --no-cpu-baseline --mesh-subdiv 0 $A > $f 2>&1 || { tail -3 $f; exit 1; }
    ba $f "$cfg $v"
  done
done
exit 0
