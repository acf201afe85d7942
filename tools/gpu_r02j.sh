#!/bin/bash
# deterministic + transfer tests, then a profiled c2 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_deterministic_gpu.py tests/test_transfer_gpu.py tests/test_ceres_surface_gpu.py tests/test_sanitize.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_r02j.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/pytest_r02j.log | head -20; tail -40 gpurun_out/pytest_r02j.log; exit 1; }
tail -2 gpurun_out/pytest_r02j.log
bash tools/gpu_prof_c2.sh r02j
python3 -c "import json;l=json.loads([x for x in open('gpurun_out/bench_r02j.log') if x.startswith('{')][-1]);print(json.dumps(l['ceres_surface']['ms']), json.dumps(l.get('ba_deterministic'),indent=1))"
