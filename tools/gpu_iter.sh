#!/bin/bash
# Short GPU iteration: GPU tests, then the c2 bench under rocprofv3 kernel
# stats (solver kernels per CG iteration). Stops at the first fault/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-iter}
CFG=${2:-c2}
run() {
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run pytest_gpu_$TAG 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread
run prof_${CFG}_$TAG 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_${CFG}_$TAG -o run --output-format csv -- python3 bench.py --config $CFG --steps 10 --no-cpu-baseline
python3 tools/bench_summary.py $OUT/prof_${CFG}_$TAG.log
exit 0
