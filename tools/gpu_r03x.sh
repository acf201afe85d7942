#!/bin/bash
# XCD-contiguous block order for the CG passes (in-tree build, MVBA_XCD_SOLVER=1)
# against the plain order (tools/ab/xcdoff, MVBA_XCD_SOLVER=0): solver tests with
# the new build, then kernel traces at c2 (x2) and c3 (x2) of both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_solver_gpu.py tests/test_solver_forms_gpu.py tests/test_deterministic_gpu.py tests/test_linearize_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_xcd.log 2>&1
rc=$?; tail -1 $OUT/pytest_xcd.log; [ $rc -eq 0 ] || exit $rc
for cfg in c2 c3 c2 c3; do
  for v in xcd plain; do
    unset MVBA_LIB; [ $v = plain ] && export MVBA_LIB=$PWD/tools/ab/xcdoff/libmvba.so
    if [ $cfg = c3 ]; then A="--config c3 --steps 3 --ba-iters 3"; else A="--steps 5 --ba-iters 5"; fi
    d=$OUT/kt_xcd_${cfg}_${v}_$RANDOM
    timeout -s KILL 300 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 bench.py $A --no-cpu-baseline --mesh-subdiv 0 > $d.log 2>&1 || { tail -3 $d.log; exit 1; }
    echo "== $cfg $v"
    python3 tools/ktrace_med.py $d/run_kernel_trace.csv | grep -E "k_pass_b|k_pass_a_frame|k_point_w|k_pass_sq|k_cg_update|k_vec_rep|k_frame_lin"
  done
done
exit 0
