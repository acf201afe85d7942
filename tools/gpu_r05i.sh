#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r05i}
timeout -k 10 300 python tools/san_cli_repro.py cur_$TAG || exit 1
timeout -k 10 300 python tools/san_cli_repro.py nos_$TAG MVBA_OWN_STREAM=0 || exit 1
timeout -k 10 400 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_solver_forms_gpu.py tests/test_sanitize.py -s > $OUT/pytest_forms_$TAG.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -4 $OUT/pytest_forms_$TAG.log; grep "residual" $OUT/pytest_forms_$TAG.log | head
