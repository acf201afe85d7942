#!/bin/bash
# Same-box A/B: the c2 bench under rocprofv3 kernel stats, alternating the
# in-tree libmvba.so with another build of the ABI (MVBA_LIB), twice each.
# usage: tools/gpu_ab.sh <other.so> [config]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
OTHER=$1
CFG=${2:-c2}
for rep in 1 2; do
  for v in base cur; do
    if [ $v = base ]; then export MVBA_LIB=$PWD/$OTHER; else unset MVBA_LIB; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ab_${v}_$rep -o run --output-format csv -- python3 bench.py --config $CFG --steps 10 --no-cpu-baseline > $OUT/ab_${v}_$rep.log 2>&1 || { echo "$v $rep failed"; tail -5 $OUT/ab_${v}_$rep.log; exit 1; }
    echo "$v $rep: $(python3 tools/bench_summary.py $OUT/ab_${v}_$rep.log)"
  done
done
