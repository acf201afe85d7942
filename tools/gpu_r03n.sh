#!/bin/bash
# Full GPU suite (small rigs with < 2 segments per frame now take k_eval_local),
# then fused/split/local evaluation A/B on rank 0's shard of 2-, 4- and 8-way
# c2 splits (MVBA_EVAL_MODE), alternated twice, with the host enqueue time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03n}
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
exit 0
