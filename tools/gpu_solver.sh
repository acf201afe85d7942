#!/bin/bash
# GPU session: solver tests, bench (no CPU baseline), rocprof stats of the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-solver}
timeout -k 10 600 python -m pytest tests/test_solver_gpu.py tests/test_linearize_gpu.py -q -x -p no:cacheprovider > $OUT/pytest_solver.log 2>&1
rc=$?; tail -3 $OUT/pytest_solver.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > $OUT/bench_$TAG.log 2>&1 || exit $?
tail -1 $OUT/bench_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d.get('ba')))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 10 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1
exit $?
