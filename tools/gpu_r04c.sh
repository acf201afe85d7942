#!/bin/bash
# Packed K1 windows: the GPU suite, then a same-box A/B against the aligned
# layout (tools/ab/base_r04c/libmvba.so, built from the previous commit).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r04.sh r04c tests || exit $?
BASE=tools/ab/base_r04c/libmvba.so bash tools/gpu_r04.sh r04c ab || exit $?
exit 0
