#!/bin/bash
# Default bench line (CPU baseline included) and rocprof kernel stats of the
# same command on the current build; then the shard rehearsal (rank 0's shard of
# an N-way split) for N = 1, 2, 4, 8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03h}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.log 2>&1 || { tail -5 $OUT/bench_$TAG.log; exit 1; }
tail -c 600 $OUT/bench_$TAG.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1 || { tail -5 $OUT/prof_$TAG.log; exit 1; }
echo "=== prof done"
for n in 1 2 4 8; do
  timeout -k 10 200 python3 bench.py --shard-of $n --steps 50 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 3 > $OUT/shard_${n}_$TAG.log 2>&1 || { echo "shard $n failed"; tail -5 $OUT/shard_${n}_$TAG.log; exit 1; }
  python3 - $OUT/shard_${n}_$TAG.log $n <<'PY'
import json,sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d=json.loads(ln); r=d["roofline"]; b=d.get("ba",{})
        print("1/%s shard: %d obs, step %.1f us (prep %.1f, K1 %.1f), x%s = %.2e evals/s; CG iteration %.1f us" % (sys.argv[2], d["config"]["num_residuals_per_gpu"], 1e3*d["ms_per_step"], 1e3*r["prep_ms"], 1e3*r["kernel_ms"], sys.argv[2], int(sys.argv[2])*d["value"], 1e3*b.get("ms_per_cg_iteration",0)))
PY
done
exit 0
