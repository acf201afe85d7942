#!/bin/bash
# CG update + frame directions fused (no k_frame_dir per CG iteration):
# solver GPU tests, then a same-box A/B of the CG iteration against the
# direction-kernel path (MVBA_CG_DIR_KERNEL=1), alternated, at c2 and c3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03d}
OUT=gpurun_out
mkdir -p $OUT
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step tests_$TAG 600 python -u -m pytest tests/test_solver_gpu.py tests/test_deterministic_gpu.py tests/test_edge_cases.py \
  tests/test_xyz_prior.py tests/test_depth.py tests/test_cli.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
for k in 1 2; do
  for v in 0 1; do
    step ab_c2_dk${v}_$k 300 env MVBA_CG_DIR_KERNEL=$v python bench.py --no-cpu-baseline --mesh-subdiv 0 --steps 5
    grep -o '"ba": {[^}]*}' $OUT/ab_c2_dk${v}_$k.log | grep -o '"cg_iterations": [0-9]*, "ms_per_cg_iteration": [0-9.]*'
    grep -o '"ba_deterministic": {[^}]*}' $OUT/ab_c2_dk${v}_$k.log | grep -o '"cg_iterations": [0-9]*, "ms_per_cg_iteration": [0-9.]*'
  done
done
for v in 0 1; do
  step ab_c3_dk${v} 500 env MVBA_CG_DIR_KERNEL=$v python bench.py --config c3 --no-cpu-baseline --mesh-subdiv 0 --steps 3 --ba-iters 3
  grep -o '"ba": {[^}]*}' $OUT/ab_c3_dk${v}.log | grep -o '"cg_iterations": [0-9]*, "ms_per_cg_iteration": [0-9.]*'
done
exit 0
