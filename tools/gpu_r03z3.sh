#!/bin/bash
# k_pass_sq block cap sweep (MVBA_SQ_GRID) with the frame-order back-substitution, c3 and c2 kernel traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03z3}
OUT=gpurun_out
mkdir -p $OUT
for cfg in c3 c2; do
  for g in 256 512 1024 2048; do
    d=$OUT/kt_${cfg}_g${g}_$TAG
    timeout -s KILL 300 env MVBA_BACKSUB=frame MVBA_SQ_GRID=$g rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 bench.py --config $cfg --steps 3 --ba-iters 3 --no-cpu-baseline --mesh-subdiv 0 > $d.log 2>&1 || { tail -3 $d.log; exit 1; }
    echo "== $cfg grid $g: $(python3 tools/ktrace_med.py $d/run_kernel_trace.csv 0 | grep k_pass_sq)"
  done
done
exit 0
