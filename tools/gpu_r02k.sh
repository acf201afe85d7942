#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_transfer_gpu.py tests/test_ceres_surface_gpu.py tests/test_parity_gpu.py tests/test_depth.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_r02k.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/pytest_r02k.log | head; tail -30 gpurun_out/pytest_r02k.log; exit 1; }
tail -1 gpurun_out/pytest_r02k.log
bash tools/gpu_rows_pmc.sh
