#!/bin/bash
# BA roofline of one CG iteration (bench ba.roofline's committed summary):
# a kernel trace of the bench's LM phase, then separate PMC passes of the same
# command (FETCH_SIZE; WRITE_SIZE; SQ wave/VALU counters; L2 hit/miss), folded
# by tools/ba_roofline.py into gpurun_out/ba_<cfg>.json.
# usage: tools/gpu_ba_roofline.sh CFG TAG [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
CFG=${1:-c2}
TAG=${2:-ba}
shift 2 || true
B="python3 bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 3 $*"
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps_$TAG.log
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc" | tee -a $OUT/steps_$TAG.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "$OUT/$name.log"; exit $rc; fi
}
D=$OUT/ba_${CFG}_$TAG
run kt_${CFG}_$TAG 400 rocprofv3 --kernel-trace -d $D/kt -o run --output-format csv -- $B
run fetch_${CFG}_$TAG 400 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run --output-format csv -- $B
run write_${CFG}_$TAG 400 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run --output-format csv -- $B
run sq_${CFG}_$TAG 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU -d $D/sq -o run --output-format csv -- $B
run l2_${CFG}_$TAG 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $D/l2 -o run --output-format csv -- $B
f() { find "$D/$1" -name "$2" | head -1; }
python3 tools/ba_roofline.py $OUT/ba_${CFG}_$TAG.json $CFG "$(f kt '*kernel_trace.csv')" \
  "$(f fetch '*counter_collection.csv')" "$(f write '*counter_collection.csv')" "$(f sq '*counter_collection.csv')" \
  "$(f l2 '*counter_collection.csv')"
