#!/bin/bash
# full GPU suite, then c3 A/B of pass B's reduction (transposed vs per-value
# wave sums, tools/ab/tred0 = -DMVBA_PASSB_TRED=0) and the CG timing split
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r05j}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -4 $OUT/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for k in 1 2; do
  for v in cur tred0; do
    if [ $v = cur ]; then unset MVBA_LIB; else export MVBA_LIB=$PWD/tools/ab/tred0/libmvba.so; fi
    D=$OUT/kt_$TAG/c3_${v}_$k
    timeout -k 10 400 rocprofv3 --kernel-trace -d $D -o run --output-format csv -- python3 bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 2 > $OUT/kt_c3_${v}_${k}_$TAG.log 2>&1 || exit 1
    f=$(find $D -name '*kernel_trace.csv' | head -1)
    python3 tools/cg_iter_med.py c3_${v}_$k $f | tee -a $OUT/cg_iter_$TAG.txt
    gzip $f
  done
done
unset MVBA_LIB
for cfg in s8 c2 c3; do
  case $cfg in s8) A="--shard-of 8 --ba-iters 5";; c2) A="--ba-iters 5";; c3) A="--config c3 --ba-iters 3 --steps 20";; esac
  MVBA_CG_TIMING=1 timeout -k 10 400 python bench.py --steps 100 --no-cpu-baseline --mesh-subdiv 0 $A > $OUT/${cfg}_$TAG.log 2>&1 || exit 1
  echo "$cfg: $(grep 'cg timing' $OUT/${cfg}_$TAG.log | tail -1 | sed 's/.*CG iterations/CG iterations/')"
  python3 tools/bench_summary.py $OUT/${cfg}_$TAG.log | tail -1
done
