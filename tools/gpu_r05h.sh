#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r05h}
timeout -k 10 300 python tools/san_cli_repro.py g1_$TAG || exit 1
timeout -k 10 300 python tools/san_cli_repro.py g0_$TAG MVBA_CG_GRAPH=0 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread --deselect tests/test_sanitize.py::test_cli_end_to_end_under_sanitizers > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -4 $OUT/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_kt_r05.sh $TAG "s8 c2" "cur=MVBA_CG_GRAPH=1 prec0=MVBA_PREC_SMALL=0" || exit 1
for cfg in s8 c2 c3; do
  case $cfg in s8) A="--shard-of 8 --ba-iters 5";; c2) A="--ba-iters 5";; c3) A="--config c3 --ba-iters 2 --steps 20";; esac
  MVBA_CG_TIMING=1 timeout -k 10 400 python bench.py --steps 100 --no-cpu-baseline --mesh-subdiv 0 $A > $OUT/${cfg}_$TAG.log 2>&1 || exit 1
  echo "$cfg: $(grep 'cg timing' $OUT/${cfg}_$TAG.log | tail -1 | sed 's/.*batches) | //')"
  python3 tools/bench_summary.py $OUT/${cfg}_$TAG.log | tail -1
done
