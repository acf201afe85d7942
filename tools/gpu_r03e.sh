#!/bin/bash
# Round-3 measurement pass on the fused-direction CG build: per config a
# rocprofv3 kernel trace of the bench (BA phase included) and separate PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ stall/issue counters, fp64 instruction counts),
# each under its own kill timer. Summaries are made on the container side
# (tools/ba_roofline.py, tools/pmc_summary.py, tools/pmc_flops.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03e}
CFGS=${CFGS:-c2 c3 c5}
OUT=gpurun_out
mkdir -p $OUT
pmc() {
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -s KILL "$secs" rocprofv3 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -1 "$OUT/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for CFG in $CFGS; do
  B="python3 bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 2"
  pmc trace_${CFG}_$TAG 240 --kernel-trace --stats -d $OUT/trace_${CFG}_$TAG -o run --output-format csv -- $B
  pmc fetch_${CFG}_$TAG 240 --pmc FETCH_SIZE -d $OUT/fetch_${CFG}_$TAG -o run --output-format csv -- $B
  pmc write_${CFG}_$TAG 240 --pmc WRITE_SIZE -d $OUT/write_${CFG}_$TAG -o run --output-format csv -- $B
  pmc sq_${CFG}_$TAG 240 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES \
    -d $OUT/sq_${CFG}_$TAG -o run --output-format csv -- $B
  pmc flops_${CFG}_$TAG 240 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVES \
    -d $OUT/flops_${CFG}_$TAG -o run --output-format csv -- $B
done
exit 0
