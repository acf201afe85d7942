#!/bin/bash
# Round 3, first measurement call of this session: GPU suite on the current
# tree, the default bench line, rocprof kernel stats of the c2 bench, then the
# solver-kernel PMC passes at c2 (FETCH_SIZE, WRITE_SIZE, SQ stall counters;
# one pass per run, each under its own kill timer). tools/pmc_solver.py
# summarises the CSVs afterwards (on the container side).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03c}
CFGS=${CFGS:-c2}
OUT=gpurun_out
mkdir -p $OUT
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -3 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
pmc() {
  local name=$1; shift
  echo "=== $name"
  timeout -s KILL 150 rocprofv3 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
if [ -z "${SKIP_TESTS:-}" ]; then
  step pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread
fi
step bench_$TAG 600 python bench.py --no-cpu-baseline
for CFG in $CFGS; do
  B="python3 bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline --mesh-subdiv 0"
  pmc kstats_${CFG}_$TAG --kernel-trace --stats -d $OUT/kstats_${CFG}_$TAG -o run --output-format csv -- $B
  pmc fetch_${CFG}_$TAG --pmc FETCH_SIZE -d $OUT/fetch_${CFG}_$TAG -o run --output-format csv -- $B --ba-iters 2
  pmc write_${CFG}_$TAG --pmc WRITE_SIZE -d $OUT/write_${CFG}_$TAG -o run --output-format csv -- $B --ba-iters 2
  pmc sq_${CFG}_$TAG --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES \
    -d $OUT/sq_${CFG}_$TAG -o run --output-format csv -- $B --ba-iters 2
done
exit 0
