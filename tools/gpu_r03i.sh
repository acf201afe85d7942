#!/bin/bash
# bench lines after gating the committed PMC summaries to the whole-config line:
# whole c2 (summaries applied), rank 0's 8-way shard and a 2-rank gloo run (null).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_c2_r03i.log 2>&1 || { tail -5 $OUT/bench_c2_r03i.log; exit 1; }
timeout -k 10 300 python bench.py --shard-of 8 --no-cpu-baseline > $OUT/bench_shard8_r03i.log 2>&1 || { tail -5 $OUT/bench_shard8_r03i.log; exit 1; }
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline > $OUT/bench_gloo2_r03i.log 2>&1 || { tail -5 $OUT/bench_gloo2_r03i.log; exit 1; }
for f in c2 shard8 gloo2; do
  python3 - $OUT/bench_${f}_r03i.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        r = d["roofline"]; b = d.get("ba") or {}
        print(sys.argv[1], "n_gpus", d["n_gpus"], "value %.3g" % d["value"], "frac %.3f" % r["frac"],
              "traffic", r["traffic"], "binding", r.get("binding"), "ba.traffic", (b.get("roofline") or {}).get("traffic"))
PY
done
