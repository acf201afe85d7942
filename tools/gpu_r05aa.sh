#!/bin/bash
# pass-B vector replicas re-measured with today's chunks (32 since round 2):
# 16 and 8 (tools/ab/rep16, rep8) against the tree, same-box kernel traces
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05aa}
REPS="1 2" bash tools/gpu_kt_r05.sh $TAG "c2 s8 c3" "cur=MVBA_CG_GRAPH=1 rep16=MVBA_LIB=$PWD/tools/ab/rep16/libmvba.so rep8=MVBA_LIB=$PWD/tools/ab/rep8/libmvba.so" || exit 1
