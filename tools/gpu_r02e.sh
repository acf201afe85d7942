#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_linearize_gpu.py tests/test_depth.py tests/test_xyz_prior.py tests/test_solver_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_r02e.log 2>&1 || { tail -30 gpurun_out/pytest_r02e.log; exit 1; }
tail -2 gpurun_out/pytest_r02e.log
bash tools/gpu_ab.sh tools/libmvba_w4.so c2
