#!/bin/bash
# r05y's timing half (its pytest gate stopped at the point-solve forms test):
# same-box kernel traces of tools/ab/po and tools/ab/pa against the tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05y}
REPS="1 2" bash tools/gpu_kt_r05.sh $TAG "c2 s8 c3" "cur=MVBA_CG_GRAPH=1 po=MVBA_LIB=$PWD/tools/ab/po/libmvba.so pa=MVBA_LIB=$PWD/tools/ab/pa/libmvba.so" || exit 1
