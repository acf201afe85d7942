#!/bin/bash
# which round-5 change moves test_depth_mesh_one_exact_step_matches_dense_lm?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
T=tests/test_mesh.py::test_depth_mesh_one_exact_step_matches_dense_lm
for v in cur w1 g0 fast0 pqgrid merged0; do
  E=""
  case $v in w1) E="MVBA_PASSB_WAVES=1";; g0) E="MVBA_CG_GRAPH=0";; pqgrid) E="MVBA_CG_PQ=grid";; merged0) E="MVBA_LM_MERGED=0";; esac
  if [ $v = fast0 ]; then export MVBA_LIB=$PWD/tools/ab/fast0/libmvba.so; else unset MVBA_LIB; fi
  env $E timeout -k 10 200 python -u -m pytest -q -p no:cacheprovider --timeout 150 --timeout-method thread $T > $OUT/mesh_${v}.log 2>&1
  echo "$v rc $? $(grep -o 'AssertionError: .*' $OUT/mesh_${v}.log | head -1 | cut -c1-80)"
done
