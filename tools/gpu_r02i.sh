#!/bin/bash
# Deterministic mode tests + the solver/linearize suites, then c2 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sanitize.py tests/test_deterministic_gpu.py tests/test_ceres_surface_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_r02i.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/pytest_r02i.log | head -20; tail -40 gpurun_out/pytest_r02i.log; exit 1; }
tail -2 gpurun_out/pytest_r02i.log
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/bench_c2_r02i.log 2>&1 || { tail -20 gpurun_out/bench_c2_r02i.log; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_c2_r02i.log
python3 -c "import json;l=json.loads([x for x in open('gpurun_out/bench_c2_r02i.log') if x.startswith('{')][-1]);print(json.dumps(l['ceres_surface'],indent=1));print(json.dumps(l.get('ba_deterministic'),indent=1))"
