#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_r02l.log 2>&1
rc=$?
grep -E "FAILED|passed|failed" gpurun_out/pytest_gpu_r02l.log | tail -8
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3_r02l -o run --output-format csv -- python3 bench.py --config c3 --steps 10 --no-cpu-baseline > gpurun_out/bench_c3_r02l.log 2>&1
echo c3 rc $?
python3 tools/bench_summary.py gpurun_out/bench_c3_r02l.log
