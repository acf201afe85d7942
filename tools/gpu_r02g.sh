#!/bin/bash
# Host hand-over (k_rows + pinned copies), Ceres adapter, RPC d>=4 solver; c2 bench with the ceres_surface line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_transfer_gpu.py tests/test_ceres_surface_gpu.py tests/test_parity_gpu.py tests/test_depth.py tests/test_solver_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_r02g.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/pytest_r02g.log | head -20; tail -30 gpurun_out/pytest_r02g.log; exit 1; }
tail -2 gpurun_out/pytest_r02g.log
timeout -k 10 300 python bench.py --steps 10 > gpurun_out/bench_c2_r02g.log 2>&1 || { tail -20 gpurun_out/bench_c2_r02g.log; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_c2_r02g.log
python3 -c "import json;l=json.loads([x for x in open('gpurun_out/bench_c2_r02g.log') if x.startswith('{')][-1]);print(json.dumps(l['ceres_surface'],indent=1))"
