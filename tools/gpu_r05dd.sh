#!/bin/bash
# replica reduction with 4 lanes per entry (tools/ab/rl4): the full GPU suite on
# the variant, then same-box kernel traces against the tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r05dd}
V=$PWD/tools/ab/rl4/libmvba.so
MVBA_LIB=$V timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread > $OUT/pytest_rl4_$TAG.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 $OUT/pytest_rl4_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
REPS="1 2" bash tools/gpu_kt_r05.sh $TAG "c2 s8 c3" "cur=MVBA_CG_GRAPH=1 rl4=MVBA_LIB=$V" || exit 1
