#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r05k}
timeout -k 10 500 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_solver_gpu.py tests/test_solver_forms_gpu.py tests/test_deterministic_gpu.py tests/test_edge_cases.py -s > $OUT/pytest_solver_$TAG.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 $OUT/pytest_solver_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_kt_r05.sh $TAG "c2 s8" "w2=MVBA_PASSB_WAVES=2 w1=MVBA_PASSB_WAVES=1" || exit 1
# same-box A/B of the FAST projection (tools/ab/fast0: -DMVBA_FAST_PROJ=0)
for v in cur fast0; do
  for cfg in c2 c3; do
    case $cfg in c2) A="--ba-iters 5";; c3) A="--config c3 --ba-iters 2";; esac
    if [ $v = cur ]; then unset MVBA_LIB; else export MVBA_LIB=$PWD/tools/ab/fast0/libmvba.so; fi
    D=$OUT/kt_$TAG/${cfg}_$v
    timeout -k 10 400 rocprofv3 --kernel-trace -d $D -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --mesh-subdiv 0 $A > $OUT/kt_${cfg}_${v}_$TAG.log 2>&1 || exit 1
    f=$(find $D -name '*kernel_trace.csv' | head -1)
    python3 tools/cg_iter_med.py ${cfg}_$v $f | tee -a $OUT/cg_iter_$TAG.txt
    gzip $f
  done
done
unset MVBA_LIB
for cfg in s8 c2; do
  case $cfg in s8) A="--shard-of 8 --ba-iters 5";; c2) A="--ba-iters 5";; esac
  for p in 1 0; do
    MVBA_CG_PIPE=$p MVBA_CG_TIMING=1 timeout -k 10 400 python bench.py --steps 100 --no-cpu-baseline --mesh-subdiv 0 $A > $OUT/${cfg}_p${p}_$TAG.log 2>&1 || exit 1
    echo "$cfg pipe=$p: $(grep 'cg timing' $OUT/${cfg}_p${p}_$TAG.log | tail -1 | sed 's/.*CG iterations/CG iterations/')"
    python3 tools/bench_summary.py $OUT/${cfg}_p${p}_$TAG.log | tail -1
  done
done
timeout -k 10 300 python tools/c3_alloc_probe.py 5 > $OUT/c3_alloc_$TAG.log 2>&1; tail -7 $OUT/c3_alloc_$TAG.log
# K2 waves per frame part: same-box A/B (tools/ab/flin1, flin4 = -DMVBA_FLIN_WAVES=1 / 4; the tree: 2)
for k in 1 2; do
  for v in cur flin1 flin4; do
    if [ $v = cur ]; then unset MVBA_LIB; else export MVBA_LIB=$PWD/tools/ab/$v/libmvba.so; fi
    timeout -k 10 300 python bench.py --steps 200 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 0 > $OUT/lin_${v}_${k}_$TAG.log 2>&1 || exit 1
    echo "lin $v $k: $(python3 -c "
import json,sys
for l in open('$OUT/lin_${v}_${k}_$TAG.log'):
    if l.startswith('{'):
        d=json.loads(l); L=d.get('linearize',{}); print('kernel_ms', round(L.get('kernel_ms',0)*1e3,1), 'records_current', round(L.get('kernel_ms_records_current',0)*1e3,1), 'mfma util', round(L.get('mfma',{}).get('util',0),3))
")"
  done
done
unset MVBA_LIB
