#!/bin/bash
# Evaluation step / prep / K1 times of the in-tree build beside variant builds
# (tools/build_variant.sh), alternated twice: tools/gpu_prep_diag.sh tools/ab/NAME ...
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/diag
for rep in 1 2; do for v in cur "$@"; do
  if [ $v = cur ]; then unset MVBA_LIB; else export MVBA_LIB=$PWD/$v/libmvba.so; fi
  tag=$(basename $v)
  timeout -k 10 200 python3 bench.py --steps 50 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 0 > gpurun_out/diag/${tag}_$rep.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/diag/${tag}_$rep.log; exit 1; }
  python3 - gpurun_out/diag/${tag}_$rep.log $tag <<'PY'
import json,sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d=json.loads(ln); print(sys.argv[2], "step %.1f us prep %.1f us K1 %.1f us" % (1e3*d["ms_per_step"], 1e3*d["roofline"]["prep_ms"], 1e3*d["roofline"]["kernel_ms"]))
PY
done; done
