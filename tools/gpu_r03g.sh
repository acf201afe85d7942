#!/bin/bash
# Fused prep + K1 (k_eval: K0 blocks hand frame records to K1 waves in one
# launch): full GPU suite, then same-box A/B against two launches
# (MVBA_SPLIT_PREP=1), alternated: c2, rank 0's 8-way shard of c2, c3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03g}
OUT=gpurun_out
mkdir -p $OUT
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log" | cut -c1-300; echo "stopping after $name (rc=$rc)"; exit $rc; fi
  tail -1 "$OUT/$name.log" | cut -c1-160
}
summ() { python3 -c "
import json,sys
for ln in open('$1'):
    if ln.startswith('{'):
        d=json.loads(ln); r=d['roofline']
        print('  value %.3e  step %.2f us  K1 %.2f us  prep %.2f us' % (d['value'], 1e3*d['ms_per_step'], 1e3*r['kernel_ms'], 1e3*r['prep_ms']))
"; }
step pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread
for k in 1 2; do
  for v in 0 1; do
    step ab_c2_sp${v}_$k 300 env MVBA_SPLIT_PREP=$v python bench.py --no-cpu-baseline --mesh-subdiv 0 --steps 50 --ba-iters 0
    summ $OUT/ab_c2_sp${v}_$k.log
    step ab_s8_sp${v}_$k 300 env MVBA_SPLIT_PREP=$v python bench.py --shard-of 8 --no-cpu-baseline --mesh-subdiv 0 --steps 50 --ba-iters 0
    summ $OUT/ab_s8_sp${v}_$k.log
  done
done
for v in 0 1; do
  step ab_c3_sp${v} 400 env MVBA_SPLIT_PREP=$v python bench.py --config c3 --no-cpu-baseline --mesh-subdiv 0 --steps 10 --ba-iters 0
  summ $OUT/ab_c3_sp${v}.log
done
exit 0
