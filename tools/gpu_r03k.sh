#!/bin/bash
# Fused vs split evaluation on rank 0's shard of a 2- and 4-way split of c2
# (MVBA_SPLIT_PREP), alternated twice, to place the fused/split threshold.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
summ() { python3 -c "
import json,sys
for ln in open('$1'):
    if ln.startswith('{'):
        d=json.loads(ln); r=d['roofline']
        print('  %s: step %.2f us  K1 %.2f us  prep %.2f us' % ('$2', 1e3*d['ms_per_step'], 1e3*r['kernel_ms'], 1e3*r['prep_ms']))
"; }
for k in 1 2; do
  for n in 2 4; do
    for v in 0 1; do
      f=$OUT/shardab_${n}_sp${v}_$k.log
      timeout -k 10 200 env MVBA_SPLIT_PREP=$v python3 bench.py --shard-of $n --steps 50 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 0 > $f 2>&1 || { tail -3 $f; exit 1; }
      summ $f "N=$n split=$v"
    done
  done
done
exit 0
