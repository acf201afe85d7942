#!/bin/bash
# Slots in landmark order within each frame (default) against AddResidualBlock
# order (MVBA_SLOT_ORDER=insertion): the whole GPU suite on the new layout, then
# kernel traces of the bench at c2 (x2) and c3 (x2) in both layouts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_slot.log 2>&1
rc=$?; tail -1 $OUT/pytest_slot.log; [ $rc -eq 0 ] || exit $rc
for cfg in c2 c3 c2 c3; do
  for v in sorted insertion; do
    unset MVBA_SLOT_ORDER; [ $v = insertion ] && export MVBA_SLOT_ORDER=insertion
    if [ $cfg = c3 ]; then A="--config c3 --steps 3 --ba-iters 3"; else A="--steps 5 --ba-iters 5"; fi
    d=$OUT/kt_slot_${cfg}_${v}_$RANDOM
    timeout -s KILL 300 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 bench.py $A --no-cpu-baseline --mesh-subdiv 0 > $d.log 2>&1 || { tail -3 $d.log; exit 1; }
    echo "== $cfg $v"
    python3 tools/ktrace_med.py $d/run_kernel_trace.csv | grep -E "k_pass_b|k_pass_a_frame|k_point_w|k_pass_sq|k_cg_update|k_frame_lin|k_eval|k_obs<"
  done
done
exit 0
