#!/bin/bash
# CG iteration A/B (same box, alternated twice): base = previous commit,
# cur = nontemporal streaming loads in the CG passes + the replica count sized
# by the chunk count, nt0 = cur without the nontemporal loads; c2, c3 and rank
# 0's 1/8 shard of c2 (bench ba.ms_per_cg_iteration), then the GPU tests that
# the last run failed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=r04d
run() {
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" >> $OUT/steps_$TAG.log
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; tail -5 $OUT/$name.log; exit $rc; fi
  return $rc
}
cg() { python3 - "$1" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d = json.loads(ln); b = d["ba"]
        print(f"{sys.argv[1].split('/')[-1]:32s} {1e3 * b['ms_per_cg_iteration']:8.1f} us/CG  ({b['cg_iterations']} CG, {b['iters_per_s']:.1f} LM it/s)")
PY
}
for k in 1 2; do
  for v in base cur nt0; do
    case $v in base) export MVBA_LIB=$PWD/tools/ab/base_r04d/libmvba.so;; nt0) export MVBA_LIB=$PWD/tools/ab/nt0_r04d/libmvba.so;; cur) unset MVBA_LIB;; esac
    run cg_c2_${v}_$k 300 python3 bench.py --steps 20 --ba-iters 5 --no-cpu-baseline --mesh-subdiv 0 && cg $OUT/cg_c2_${v}_$k.log
    run cg_s8_${v}_$k 300 python3 bench.py --shard-of 8 --steps 20 --ba-iters 5 --no-cpu-baseline --mesh-subdiv 0 && cg $OUT/cg_s8_${v}_$k.log
    run cg_c3_${v}_$k 400 python3 bench.py --config c3 --steps 5 --ba-iters 4 --no-cpu-baseline --mesh-subdiv 0 && cg $OUT/cg_c3_${v}_$k.log
  done
done
unset MVBA_LIB
run pytest_$TAG 600 python -u -m pytest tests/test_bench_failure_gpu.py tests/test_solver_forms_gpu.py tests/test_eval_forms_gpu.py tests/test_solver_gpu.py tests/test_deterministic_gpu.py -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread
tail -3 $OUT/pytest_$TAG.log
exit 0
