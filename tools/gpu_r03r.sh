#!/bin/bash
# K1 with two waves per segment in the thin-shard evaluation (MVBA_K1_SPLIT=1):
# parity tests with it forced on, then rank 0's shard of 8-, 4-, 2-way c2
# splits, off/on alternated twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03r}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 env MVBA_K1_SPLIT=1 python -u -m pytest tests/test_parity_gpu.py tests/test_full_size_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_split_$TAG.log 2>&1
rc=$?; tail -2 $OUT/pytest_split_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_split_$TAG.log | head; exit $rc; }
summ() { python3 -c "
import json,sys
for ln in open('$1'):
    if ln.startswith('{'):
        d=json.loads(ln); r=d['roofline']
        print('  %s: step %.2f us  host enqueue %.2f us' % ('$2', 1e3*d['ms_per_step'], 1e3*d['host_issue_ms_per_step']))
"; }
for k in 1 2; do
  for n in 8 4 2; do
    for v in 0 1; do
      f=$OUT/k1split_${n}_${v}_${k}_$TAG.log
      timeout -k 10 200 env MVBA_K1_SPLIT=$v python3 bench.py --shard-of $n --steps 200 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 0 > $f 2>&1 || { tail -3 $f; exit 1; }
      summ $f "N=$n split2=$v"
    done
  done
done
exit 0
