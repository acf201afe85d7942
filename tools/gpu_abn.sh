#!/bin/bash
# Same-box A/B/..: the c2 bench (no profiler) alternating the in-tree
# libmvba.so ("cur") with other builds of the ABI loaded through MVBA_LIB,
# twice each. usage: tools/gpu_abn.sh CONFIG LIB1 [LIB2 ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/abn
mkdir -p $OUT
CFG=$1; shift
for rep in 1 2; do
  for v in cur "$@"; do
    tag=$(echo $v | tr '/' '_')
    if [ $v = cur ]; then unset MVBA_LIB; else export MVBA_LIB=$PWD/$v; fi
    timeout -k 10 300 python3 bench.py --config $CFG --steps 20 --no-cpu-baseline --mesh-subdiv 0 > $OUT/${tag}_$rep.log 2>&1 || { echo "$v $rep failed"; tail -5 $OUT/${tag}_$rep.log; exit 1; }
    echo "$v $rep: $(python3 tools/bench_summary.py $OUT/${tag}_$rep.log)"
    python3 - $OUT/${tag}_$rep.log <<'PY'
import json,sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d=json.loads(ln); L=d.get("linearize",{})
        print("    step %.1f us, prep %.1f us | lin kernel %.1f us, camera side %.1f us, point side %.1f us" % (1e3*d["ms_per_step"], 1e3*d["roofline"].get("prep_ms",0), 1e3*L.get("kernel_ms",0), 1e3*L.get("camera_side_ms",0), 1e3*L.get("point_side_ms",0)))
PY
  done
done
