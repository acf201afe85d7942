#!/bin/bash
# K2 diagnostic variants (tools/build_variant.sh with -DMVBA_FLIN_DIAG=1/2/3:
# no atomics / no MFMA / no epilogue): linearization camera-side times beside
# the in-tree build, alternated twice. Timing only: the variants' outputs are wrong.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lindiag
for rep in 1 2; do for v in cur "$@"; do
  if [ $v = cur ]; then unset MVBA_LIB; else export MVBA_LIB=$PWD/$v/libmvba.so; fi
  tag=$(basename $v)
  timeout -k 10 200 python3 bench.py --steps 10 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 0 > gpurun_out/lindiag/${tag}_$rep.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/lindiag/${tag}_$rep.log; exit 1; }
  python3 - gpurun_out/lindiag/${tag}_$rep.log $tag <<'PY'
import json,sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d=json.loads(ln); L=d["linearize"]
        print(sys.argv[2], "lin %.1f us camera side %.1f us point side %.1f us" % (1e3*L["kernel_ms"], 1e3*L.get("camera_side_ms",0), 1e3*L.get("point_side_ms",0)))
PY
done; done
