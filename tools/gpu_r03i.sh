#!/bin/bash
# k_point_w loads its point data before the c_o gathers; pass A takes two
# segments per wave with the next one's loads prefetched. Solver GPU tests,
# then same-box A/B: base (previous commit's library through MVBA_LIB), new with
# MVBA_PASS_A_PIPE=1 (point_w change only), new (both), at c2 (x2) and c3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03i}
OUT=gpurun_out
mkdir -p $OUT
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log" | cut -c1-300; echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
cg() { grep -o "\"$2\": {[^}]*}" $1 | grep -o '"cg_iterations": [0-9]*, "ms_per_cg_iteration": [0-9.]*'; }
step tests_$TAG 600 python -u -m pytest tests/test_solver_gpu.py tests/test_deterministic_gpu.py tests/test_edge_cases.py \
  tests/test_xyz_prior.py tests/test_depth.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
tail -1 $OUT/tests_$TAG.log
for cfg in c2 c2 c3; do
  for v in base pipe1 pipe2; do
    case $v in
      base) E="MVBA_LIB=tools/ab/base/libmvba.so" ;;
      pipe1) E="MVBA_PASS_A_PIPE=1" ;;
      pipe2) E="MVBA_PASS_A_PIPE=2" ;;
    esac
    n=ab_${cfg}_${v}_$RANDOM
    if [ $cfg = c3 ]; then A="--config c3 --steps 3 --ba-iters 3"; else A="--steps 5"; fi
    step $n 500 env $E python bench.py --no-cpu-baseline --mesh-subdiv 0 $A
    echo "$cfg $v: $(cg $OUT/$n.log ba) | det $(cg $OUT/$n.log ba_deterministic)"
  done
done
exit 0
