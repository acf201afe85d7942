#!/bin/bash
# Fused pass A (MVBA_FUSE_POINT_W=1): solver + deterministic tests with it on,
# then the same-box A/B of the switch on the c2 solve.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
MVBA_FUSE_POINT_W=1 timeout -k 10 400 python -u -m pytest tests/test_solver_gpu.py tests/test_deterministic_gpu.py tests/test_xyz_prior.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_fuse_w.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_fuse_w.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_env.sh MVBA_FUSE_POINT_W c2
