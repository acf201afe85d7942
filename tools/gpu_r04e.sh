#!/bin/bash
# Thin-shard K1 diagnosis (rank 0's 1/8 shard of c2): kernel trace of the
# evaluation forms, then SQ counters (waves, busy, wait, VALU) per kernel; and
# the two GPU tests fixed since the last run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=r04e
run() {
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps_$TAG.log
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc" | tee -a $OUT/steps_$TAG.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; tail -5 $OUT/$name.log; exit $rc; fi
  return $rc
}
run pytest_$TAG 600 python -u -m pytest tests/test_bench_failure_gpu.py tests/test_solver_forms_gpu.py -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread
tail -3 $OUT/pytest_$TAG.log
B="python3 bench.py --shard-of 8 --steps 200 --ba-iters 0 --no-cpu-baseline --mesh-subdiv 0"
run kt_s8_$TAG 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_s8_$TAG -o run --output-format csv -- $B
python3 tools/ktrace_med.py $OUT/kt_s8_$TAG/run_kernel_trace.csv 2 | head -20
run sq_s8_$TAG 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/sq_s8_$TAG -o run --output-format csv -- $B --steps 20
run wr_s8_$TAG 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/wr_s8_$TAG -o run --output-format csv -- $B --steps 20
B1="python3 bench.py --steps 200 --ba-iters 0 --no-cpu-baseline --mesh-subdiv 0"
run sq_c2_$TAG 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/sq_c2_$TAG -o run --output-format csv -- $B1 --steps 20
exit 0
