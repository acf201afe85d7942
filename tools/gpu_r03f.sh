#!/bin/bash
# w_p pushed into the observation slots (k_point_w -> pass B) and CG frame
# blocks without CgEntry loads: solver GPU tests, then same-box A/B against the
# wbuf[pid] gather (MVBA_W_GATHER=1), alternated, c2 twice and c3 once each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03f}
OUT=gpurun_out
mkdir -p $OUT
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log" | cut -c1-300; echo "stopping after $name (rc=$rc)"; exit $rc; fi
  tail -1 "$OUT/$name.log" | cut -c1-200
}
step tests_$TAG 600 python -u -m pytest tests/test_solver_gpu.py tests/test_deterministic_gpu.py tests/test_edge_cases.py \
  tests/test_xyz_prior.py tests/test_depth.py tests/test_cli.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
for k in 1 2; do
  for v in 0 1; do
    step ab_c2_wg${v}_$k 300 env MVBA_W_GATHER=$v python bench.py --no-cpu-baseline --mesh-subdiv 0 --steps 5
    grep -o '"ba": {[^}]*}' $OUT/ab_c2_wg${v}_$k.log | grep -o '"cg_iterations": [0-9]*, "ms_per_cg_iteration": [0-9.]*'
    grep -o '"ba_deterministic": {[^}]*}' $OUT/ab_c2_wg${v}_$k.log | grep -o '"cg_iterations": [0-9]*, "ms_per_cg_iteration": [0-9.]*'
  done
done
for v in 0 1; do
  step ab_c3_wg${v} 500 env MVBA_W_GATHER=$v python bench.py --config c3 --no-cpu-baseline --mesh-subdiv 0 --steps 3 --ba-iters 3
  grep -o '"ba": {[^}]*}' $OUT/ab_c3_wg${v}.log | grep -o '"cg_iterations": [0-9]*, "ms_per_cg_iteration": [0-9.]*'
  grep -o '"ba_deterministic": {[^}]*}' $OUT/ab_c3_wg${v}.log | grep -o '"cg_iterations": [0-9]*, "ms_per_cg_iteration": [0-9.]*'
done
B="python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 2"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_c3_$TAG -o run --output-format csv -- $B > $OUT/trace_c3_$TAG.log 2>&1 || exit $?
echo "=== trace done"
exit 0
