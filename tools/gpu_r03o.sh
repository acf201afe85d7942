#!/bin/bash
# Full GPU suite; fused/split/local evaluation A/B on rank 0's shard of 2-, 4-,
# 8-way c2 splits (MVBA_EVAL_MODE), twice; then the CG passes with direct chunk
# records against the previous build (tools/ab/base through MVBA_LIB): kernel
# traces at c2 (twice) and c3, per-kernel medians (tools/ktrace_med.py);
# 'slot': pass A stores c_o in slot order and k_point_w gathers (MVBA_CO_ORDER).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03o}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_gpu_$TAG.log | head; exit $rc; }
summ() { python3 -c "
import json,sys
for ln in open('$1'):
    if ln.startswith('{'):
        d=json.loads(ln); r=d['roofline']
        print('  %s: step %.2f us  host enqueue %.2f us  K1 %.2f us  prep %.2f us' % ('$2', 1e3*d['ms_per_step'], 1e3*d['host_issue_ms_per_step'], 1e3*r['kernel_ms'], 1e3*r['prep_ms']))
"; }
for k in 1 2; do
  for n in 8 4 2; do
    for v in split local fused; do
      f=$OUT/evm_${n}_${v}_$k.log
      timeout -k 10 200 env MVBA_EVAL_MODE=$v python3 bench.py --shard-of $n --steps 200 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 0 > $f 2>&1 || { tail -3 $f; exit 1; }
      summ $f "N=$n $v"
    done
  done
done
for cfg in c2 c2 c3; do
  for v in base cur slot; do
    unset MVBA_CO_ORDER
    if [ $v = base ]; then export MVBA_LIB=$PWD/tools/ab/base/libmvba.so; else unset MVBA_LIB; fi
    if [ $v = slot ]; then export MVBA_CO_ORDER=slot; fi
    if [ $cfg = c3 ]; then A="--config c3 --steps 3 --ba-iters 3"; else A="--steps 5 --ba-iters 5"; fi
    d=$OUT/kt_${cfg}_${v}_$RANDOM
    timeout -s KILL 300 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 bench.py --no-cpu-baseline --mesh-subdiv 0 $A > $d.log 2>&1 || { tail -3 $d.log; exit 1; }
    echo "== $cfg $v $(grep -o "\"cg_iterations\": [0-9]*, \"ms_per_cg_iteration\": [0-9.]*" $d.log | head -1)"; python3 tools/ktrace_med.py $d/run_kernel_trace.csv
  done
done
exit 0
