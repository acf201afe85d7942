#!/bin/bash
# The eval-forms test with stale records before every form: against the
# previous build (tools/ab/oldlocal: k_eval_local's inactive lanes left part of
# the frame record unstored; expected to FAIL) and the fixed in-tree build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== previous build (expected to fail)"
timeout -k 10 300 env MVBA_LIB=$PWD/tools/ab/oldlocal/libmvba.so python -u -m pytest tests/test_eval_forms_gpu.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/evalforms_old.log 2>&1
echo "rc=$?"; grep -E "passed|failed" gpurun_out/evalforms_old.log | tail -1
echo "== fixed build"
timeout -k 10 600 python -u -m pytest tests/test_eval_forms_gpu.py tests/test_depth.py tests/test_parity_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/evalforms_new.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/evalforms_new.log | tail -1; exit $rc
