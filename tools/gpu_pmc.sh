#!/bin/bash
# PMC evidence of the tree, per config (default c2 c3 c4 c5):
#  * fp64 instruction counts per kernel (one SQ pass) -> pmc_flops_<cfg>.json:
#    the headline launch's second roofline (roofline.fp64_frac / binding) and
#    the linearization's fp64_frac;
#  * FETCH_SIZE / WRITE_SIZE (separate passes) -> pmc_eval_<cfg>.json (the
#    one-launch evaluation the timed loop runs), pmc_k1_<cfg>.json (split K1),
#    and for depth configs pmc_depth_<cfg>.json (K1-depth, k_depth_obs<double>).
# Each pass its own process under a hard time limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-r05p}
run() {
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps_$TAG.log
  timeout -s KILL "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc" | tee -a $OUT/steps_$TAG.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -3 "$OUT/$name.log"; exit $rc; fi
}
for CFG in ${PMC_CFGS:-c2 c3 c4 c5}; do
  case $CFG in c4) EX="--steps 3 --warmup 1";; c3) EX="--steps 4 --warmup 1";; *) EX="--steps 5 --warmup 1";; esac
  B="python3 bench.py --config $CFG $EX --no-cpu-baseline --mesh-subdiv 0"
  D=$OUT/pmc_$TAG/$CFG
  run flops_${CFG}_$TAG 400 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVES -d $D/flops -o run --output-format csv -- $B --ba-iters 1
  run fetch_${CFG}_$TAG 400 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run --output-format csv -- $B --ba-iters 0
  run write_${CFG}_$TAG 400 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run --output-format csv -- $B --ba-iters 0
  F=$(find $D/flops -name '*counter_collection.csv' | head -1)
  FE=$(find $D/fetch -name '*counter_collection.csv' | head -1)
  WR=$(find $D/write -name '*counter_collection.csv' | head -1)
  python3 tools/pmc_flops.py $F $OUT/pmc_flops_${CFG}.json $CFG
  DEG=$(python3 -c "import sys; sys.path.insert(0, '.'); from multiview_amd import rig; from bench import kernel_degree; print(kernel_degree(rig.CONFIGS['$CFG']['models'][0]))")
  # (c4 takes the split form: no k_eval_local launch in its timed loop)
  python3 tools/pmc_summary.py $FE $WR "k_eval_local<$DEG, double, true>" $OUT/pmc_eval_${CFG}.json $CFG || echo "no k_eval_local summary for $CFG"
  python3 tools/pmc_summary.py $FE $WR "k_obs<$DEG, double>" $OUT/pmc_k1_${CFG}.json $CFG
  if [ $CFG = c5 ]; then
    python3 tools/pmc_summary.py $FE $WR "k_depth_obs<double>" $OUT/pmc_depth_${CFG}.json $CFG
  fi
  find $D -name '*.csv' -size +2M -exec gzip {} \;
done
exit 0
