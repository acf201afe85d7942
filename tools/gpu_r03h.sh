#!/bin/bash
# CG update with batched block-row loads: solver GPU tests, then same-box c2 A/B
# against the previous build (ab_base/libmvba_base.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_solver_gpu.py tests/test_deterministic_gpu.py > $OUT/pytest_solver_r03h.log 2>&1
rc=$?; tail -3 $OUT/pytest_solver_r03h.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh ab_base/libmvba_base.so c2
