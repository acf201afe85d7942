#!/bin/bash
# pipelined pass-B gathers for the non-RPC models + the first slot records of
# pass A before the direction staging (tools/ab/po), pass A alone (tools/ab/pa):
# solver tests on po, then same-box kernel traces against the tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r05y}
PO=$PWD/tools/ab/po/libmvba.so
PA=$PWD/tools/ab/pa/libmvba.so
MVBA_LIB=$PO timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_solver_gpu.py tests/test_solver_forms_gpu.py -m gpu > $OUT/pytest_po_$TAG.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 $OUT/pytest_po_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
REPS="1 2" bash tools/gpu_kt_r05.sh $TAG "c2 s8 c3" "cur=MVBA_CG_GRAPH=1 po=MVBA_LIB=$PO pa=MVBA_LIB=$PA" || exit 1
