#!/bin/bash
# Diagnostic: K1 alone (event-timed instrumented steps) with its occupancy capped
# at 3 waves per SIMD through padded dynamic LDS (MVBA_K1_LDS_PAD=49152), as the
# fused evaluation's K0-sized register file caps it, against the uncapped K1;
# c2 and c3.
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
        print('  %s: fused step %.1f us, K1 alone %.1f us' % ('$2', 1e3*d['ms_per_step'], 1e3*r['kernel_ms']))
"; }
for cfg in c2 c3; do
  for pad in 0 49152; do
    if [ $cfg = c3 ]; then A="--config c3 --steps 10"; else A="--steps 100"; fi
    f=$OUT/k1pad_${cfg}_$pad.log
    timeout -k 10 300 env MVBA_K1_LDS_PAD=$pad python3 bench.py $A --no-cpu-baseline --mesh-subdiv 0 --ba-iters 0 > $f 2>&1 || { tail -3 $f; exit 1; }
    summ $f "$cfg pad=$pad"
  done
done
exit 0
