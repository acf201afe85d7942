#!/bin/bash
# Per-rank step time of the strong-scaling headline, rehearsed in ONE process on
# one GPU: rank 0's shard of an N-way landmark split of c2 (bench.py --shard-of N).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/shard
for n in 1 2 4 8; do
  timeout -k 10 200 python3 bench.py --shard-of $n --steps 50 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 3 > gpurun_out/shard/shard_$n.log 2>&1 || { echo "shard $n failed"; tail -5 gpurun_out/shard/shard_$n.log; exit 1; }
  python3 - gpurun_out/shard/shard_$n.log $n <<'PY'
import json,sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d=json.loads(ln); r=d["roofline"]; b=d.get("ba",{})
        sf=r["split_form"]
        print("1/%s shard: %d obs, step %.1f us (%s %.1f us; split form prep %.1f + K1 %.1f), x%s = %.2e evals/s if ranks overlap perfectly; CG iteration %.1f us" % (sys.argv[2], d["config"]["num_residuals_per_gpu"], 1e3*d["ms_per_step"], r["kernel"], 1e3*r["kernel_ms"], 1e3*sf["prep_ms"], 1e3*sf["kernel_ms"], sys.argv[2], int(sys.argv[2])*d["value"], 1e3*b.get("ms_per_cg_iteration",0)))
PY
done
