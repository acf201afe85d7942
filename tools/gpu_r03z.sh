#!/bin/bash
# Back-substitution forms at kernel level: c3 and c2 kernel traces with the
# point-order pass (default) and MVBA_BACKSUB=frame (frame-order pass A +
# k_point_w + k_pass_sq); solver tests with the frame form forced on first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03z}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 env MVBA_BACKSUB=frame python -u -m pytest tests/test_solver_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?; tail -2 $OUT/pytest_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_$TAG.log | head; exit $rc; }
for cfg in c3 c2; do
  for v in point frame; do
    d=$OUT/kt_${cfg}_${v}_$TAG
    timeout -s KILL 300 env MVBA_BACKSUB=$v rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 bench.py --config $cfg --steps 3 --ba-iters 3 --no-cpu-baseline --mesh-subdiv 0 > $d.log 2>&1 || { tail -3 $d.log; exit 1; }
    echo "== $cfg $v: $(python3 tools/bench_summary.py $d.log | grep -o 'LM.*')"
    python3 tools/ktrace_med.py $d/run_kernel_trace.csv 0 | grep -E "k_pass_a|k_point_w|k_pass_sq|k_block_prec"
  done
done
exit 0
