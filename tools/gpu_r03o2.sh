#!/bin/bash
# Software-pipelined pass B (tools/ab/pbpipe, MVBA_PASSB_PIPE=1) against the
# in-tree build: solver tests with it, then kernel traces at c2 (x2) and c3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 env MVBA_LIB=$PWD/tools/ab/pbpipe/libmvba.so python -u -m pytest tests/test_solver_gpu.py tests/test_solver_forms_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_pbpipe.log 2>&1
rc=$?; tail -1 $OUT/pytest_pbpipe.log; [ $rc -eq 0 ] || exit $rc
for cfg in c2 c2 c3; do
  for v in base pipe; do
    unset MVBA_LIB; [ $v = pipe ] && export MVBA_LIB=$PWD/tools/ab/pbpipe/libmvba.so
    if [ $cfg = c3 ]; then A="--config c3 --steps 3 --ba-iters 3"; else A="--steps 5 --ba-iters 5"; fi
    d=$OUT/kt_pb_${cfg}_${v}_$RANDOM
    timeout -s KILL 300 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 bench.py $A --no-cpu-baseline --mesh-subdiv 0 > $d.log 2>&1 || { tail -3 $d.log; exit 1; }
    echo "== $cfg $v: $(python3 tools/ktrace_med.py $d/run_kernel_trace.csv | grep k_pass_b)"
  done
done
exit 0
