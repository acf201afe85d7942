#!/bin/bash
# Software-pipelined gathers in pass B (RPC) and pass A (chunked): solver
# tests on tools/ab/pipe, then same-box kernel traces against the tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r05v}
V=$PWD/tools/ab/pipe/libmvba.so
MVBA_LIB=$V timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_solver_gpu.py tests/test_solver_forms_gpu.py -m gpu -k "rpc or forms or exact" > $OUT/pytest_pipe_$TAG.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 $OUT/pytest_pipe_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
REPS="1 2" bash tools/gpu_kt_r05.sh $TAG "c3 c2" "cur=MVBA_CG_GRAPH=1 pipe=MVBA_LIB=$V" || exit 1
