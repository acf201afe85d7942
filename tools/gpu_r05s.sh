#!/bin/bash
# r05r continued (its pytest stopped at the mesh test's own assertion): the
# rest of the solver tests on tools/ab/rf1, then the kernel traces and LM timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r05s}
RF=$PWD/tools/ab/rf1/libmvba.so
MVBA_LIB=$RF timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_mesh.py tests/test_edge_cases.py tests/test_depth.py tests/test_xyz_prior.py tests/test_fp32_eval.py -m gpu > $OUT/pytest_rf1_$TAG.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 $OUT/pytest_rf1_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_kt_r05.sh $TAG "c2 s8" "cur=MVBA_CG_GRAPH=1 rf1=MVBA_LIB=$RF" || exit 1
for cfg in s8 c2; do
  case $cfg in s8) A="--shard-of 8 --ba-iters 5";; c2) A="--ba-iters 5";; esac
  for v in cur rf1; do
    if [ $v = cur ]; then unset MVBA_LIB; else export MVBA_LIB=$RF; fi
    MVBA_CG_TIMING=1 timeout -k 10 400 python bench.py --steps 100 --no-cpu-baseline --mesh-subdiv 0 $A > $OUT/${cfg}_${v}_$TAG.log 2>&1 || exit 1
    echo "$cfg $v: $(grep 'cg timing' $OUT/${cfg}_${v}_$TAG.log | tail -1 | sed 's/.*CG iterations/CG iterations/')"
    python3 tools/bench_summary.py $OUT/${cfg}_${v}_$TAG.log | tail -1
  done
done
unset MVBA_LIB
