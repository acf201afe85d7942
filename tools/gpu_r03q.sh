#!/bin/bash
# Round-3 evidence on the current build: full GPU suite, smoke, default bench
# line (CPU baseline included) and rocprofv3 kernel stats of the same command
# (tools/gpu_final.sh); rank 0's shard of an N-way split for N = 1, 2, 4, 8;
# the c3 line and a c3 kernel trace (per-kernel medians).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03q}
OUT=gpurun_out
bash tools/gpu_final.sh $TAG || exit $?
for n in 1 2 4 8; do
  timeout -k 10 200 python3 bench.py --shard-of $n --steps 50 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 3 > $OUT/shard_${n}_$TAG.log 2>&1 || { echo "shard $n failed"; tail -5 $OUT/shard_${n}_$TAG.log; exit 1; }
  python3 - $OUT/shard_${n}_$TAG.log $n <<'PY'
import json,sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d=json.loads(ln); r=d["roofline"]; b=d.get("ba",{})
        print("1/%s shard: %d obs, step %.1f us (host enqueue %.1f; prep %.1f, K1 %.1f event-timed), x%s = %.2e evals/s; CG iteration %.1f us" % (sys.argv[2], d["config"]["num_residuals_per_gpu"], 1e3*d["ms_per_step"], 1e3*d["host_issue_ms_per_step"], 1e3*r["prep_ms"], 1e3*r["kernel_ms"], sys.argv[2], int(sys.argv[2])*d["value"], 1e3*b.get("ms_per_cg_iteration",0)))
PY
done
timeout -k 10 400 python3 bench.py --config c3 --steps 3 --ba-iters 3 --no-cpu-baseline > $OUT/bench_c3_$TAG.log 2>&1 || { tail -5 $OUT/bench_c3_$TAG.log; exit 1; }
python3 tools/bench_summary.py $OUT/bench_c3_$TAG.log
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3_$TAG -o run --output-format csv -- python3 bench.py --config c3 --steps 3 --ba-iters 3 --no-cpu-baseline --mesh-subdiv 0 > $OUT/prof_c3_$TAG.log 2>&1 || { tail -3 $OUT/prof_c3_$TAG.log; exit 1; }
python3 tools/ktrace_med.py $OUT/prof_c3_$TAG/run_kernel_trace.csv
exit 0
