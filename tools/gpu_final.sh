#!/bin/bash
# Round-end style evidence: the full GPU suite, smoke(), the default bench line
# and its rocprofv3 kernel stats. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-final}
OUT=gpurun_out
mkdir -p $OUT
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -3 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread
step smoke_$TAG 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_$TAG 600 python bench.py
python3 tools/bench_summary.py $OUT/bench_$TAG.log
step prof_$TAG 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 10 --no-cpu-baseline
exit 0
