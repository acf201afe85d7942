#!/bin/bash
# Round-end style evidence on the current build (full GPU suite, smoke, default
# bench line, rocprofv3 kernel stats), then rank 0's shard of an 8-way split
# with the host's enqueue time per step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03m}
bash tools/gpu_final.sh $TAG || exit $?
OUT=gpurun_out
for n in 8 1; do
  timeout -k 10 200 python3 bench.py --shard-of $n --steps 200 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 0 > $OUT/shard_${n}_$TAG.log 2>&1 || { tail -5 $OUT/shard_${n}_$TAG.log; exit 1; }
  python3 - $OUT/shard_${n}_$TAG.log $n <<'PY'
import json,sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d=json.loads(ln); r=d["roofline"]
        print("1/%s shard: step %.1f us, host enqueue %.1f us per step (prep %.1f, K1 %.1f event-timed)" % (sys.argv[2], 1e3*d["ms_per_step"], 1e3*d["host_issue_ms_per_step"], 1e3*r["prep_ms"], 1e3*r["kernel_ms"]))
PY
done
exit 0
