#!/bin/bash
# Round-3 first session: GPU suite on the round-2 kernels + ADVICE fixes, the
# self-launching multi-rank bench (gloo, 2 ranks on one GPU), the edge-case
# solve repeated in atomic and deterministic mode, the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03a}
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
step edge_repeat_$TAG 300 python tools/edge_repeat.py 4
step bench_gloo2_$TAG 600 python bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline --mesh-subdiv 0
step bench_$TAG 600 python bench.py --no-cpu-baseline
exit 0
