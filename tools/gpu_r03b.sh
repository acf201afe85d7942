#!/bin/bash
# Edge-case solve with the solver trace; the Ceres-surface tests (reference-signature factories).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
MVBA_SOLVER_TRACE=1 timeout -k 10 300 python tools/edge_repeat.py 1 > $OUT/edge_trace_r03b.log 2>&1 || exit $?
tail -5 $OUT/edge_trace_r03b.log | cut -c1-200
timeout -k 10 300 python -u -m pytest tests/test_ceres_surface_gpu.py tests/test_sanitize.py -m gpu -q -p no:cacheprovider --timeout 250 --timeout-method thread > $OUT/pytest_ceres_r03b.log 2>&1
rc=$?
tail -15 $OUT/pytest_ceres_r03b.log
exit $rc
