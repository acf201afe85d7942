#!/bin/bash
# Solver-form tests (c_o order bit-identical, back-substitution forms agree) and the eval-form tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_solver_forms_gpu.py tests/test_eval_forms_gpu.py tests/test_solver_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_forms.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/pytest_forms.log | tail -12; exit $rc
