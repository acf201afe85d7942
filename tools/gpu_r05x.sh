#!/bin/bash
# RPC pass B at 4 waves per SIMD (launch bounds; 128 VGPRs with 84 / 40 B of
# spills, with / without the pipelined gathers) against the tree (157 VGPRs,
# 3 waves): same-box c3 kernel traces, two runs each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05x}
REPS="1 2" bash tools/gpu_kt_r05.sh $TAG "c3" "cur=MVBA_CG_GRAPH=1 w4=MVBA_LIB=$PWD/tools/ab/w4/libmvba.so w4np=MVBA_LIB=$PWD/tools/ab/w4np/libmvba.so" || exit 1
