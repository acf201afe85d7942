#!/bin/bash
# Final round-3 evidence on the XCD-order / landmark-ordered-slot build: the GPU
# suite, smoke, the default bench (c2, CPU baseline included), c3 at the default
# 5 LM iterations, the one-GPU shard rehearsal and a kernel-stats profile of c2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03f4}
OUT=gpurun_out
mkdir -p $OUT
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log" | cut -c1-300; echo "stopping after $name (rc=$rc)"; exit $rc; fi
  tail -1 "$OUT/$name.log" | cut -c1-300
}
step pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke_$TAG 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_$TAG 600 python bench.py
step bench_c3_$TAG 500 python bench.py --config c3 --steps 3 --no-cpu-baseline --mesh-subdiv 0
step shard_$TAG 900 bash tools/gpu_shard_rehearsal.sh
cat $OUT/shard_$TAG.log
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 10 --no-cpu-baseline --mesh-subdiv 0 > $OUT/bench_under_rocprof_$TAG.log 2>&1 || exit $?
echo "=== profile done"
exit 0
