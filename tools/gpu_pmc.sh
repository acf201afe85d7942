#!/bin/bash
# PMC evidence for the current kernels at one config: fp64 instruction counts
# per kernel (tools/pmc_flops.py -> pmc_flops_<cfg>.json, read by bench.py for
# the second roofline), K1's HBM traffic from FETCH_SIZE / WRITE_SIZE (separate
# passes on gfx950; tools/pmc_summary.py -> pmc_k1_<cfg>.json), then the
# default bench line. Each pass in its own process under a hard time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-pmc}
CFG=${2:-c2}
K1=${3:-'k_obs<2, 0, double>'}
run() {
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -s KILL "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc" | tee -a $OUT/steps.log
  tail -2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
B="python3 bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline"
run flops_${CFG}_$TAG 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVES -d $OUT/flops_${CFG}_$TAG -o run --output-format csv -- $B --ba-iters 2
python3 tools/pmc_flops.py $OUT/flops_${CFG}_$TAG/run_counter_collection.csv $OUT/pmc_flops_${CFG}.json $CFG
run fetch_${CFG}_$TAG 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_${CFG}_$TAG -o run --output-format csv -- $B --ba-iters 0
run write_${CFG}_$TAG 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write_${CFG}_$TAG -o run --output-format csv -- $B --ba-iters 0
python3 tools/pmc_summary.py $OUT/fetch_${CFG}_$TAG/run_counter_collection.csv $OUT/write_${CFG}_$TAG/run_counter_collection.csv "$K1" $OUT/pmc_k1_${CFG}.json $CFG
exit 0
