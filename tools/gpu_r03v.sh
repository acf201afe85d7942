#!/bin/bash
# Division-free Gauss-Jordan for preconditioner blocks wider than 16: solver
# tests (incl. RPC degree 4-6 exact steps), then a c3 kernel trace (per-kernel
# medians; k_block_prec was 288 us at c3 on r03q).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03v}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_solver_gpu.py tests/test_edge_cases.py tests/test_deterministic_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?; tail -2 $OUT/pytest_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_$TAG.log | head; exit $rc; }
for cfg in c2 c3; do A="--config $cfg --steps 3 --ba-iters 3"; timeout -s KILL 300 rocprofv3 --kernel-trace -d $OUT/kt_${cfg}_$TAG -o run --output-format csv -- python3 bench.py $A --no-cpu-baseline --mesh-subdiv 0 > $OUT/kt_${cfg}_$TAG.log 2>&1 || { tail -3 $OUT/kt_${cfg}_$TAG.log; exit 1; }
python3 tools/bench_summary.py $OUT/kt_${cfg}_$TAG.log
python3 tools/ktrace_med.py $OUT/kt_${cfg}_$TAG/run_kernel_trace.csv; done
exit 0
