#!/bin/bash
# Round-5 evidence session: GPU tests, smoke, the default bench line (c2, CPU
# baseline), c1 and c3 lines, and a rocprofv3 kernel-trace summary of the c2
# bench whose k_eval average the line's roofline.kernel_ms must match.
# Each GPU step has its own time limit; the script stops at the first fault,
# abort, segfault, timeout or hang (exit codes other than 0 and pytest's 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-r05}
STEPS=${2:-all}
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps_$TAG.log
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc" | tee -a $OUT/steps_$TAG.log
  tail -4 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
if [ "$STEPS" = all ] || [ "$STEPS" = tests ]; then
  run pytest_gpu_$TAG 900 python -u -m pytest ${TESTS:-tests} -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread
  run smoke_$TAG 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$STEPS" = all ] || [ "$STEPS" = bench ]; then
  run bench_$TAG 600 python bench.py
  run bench_c1_$TAG 300 python bench.py --config c1 --mesh-subdiv 0
  run bench_c3_$TAG 600 python bench.py --config c3 --steps 50 --mesh-subdiv 0 --cpu-sample 200000
  run prof_c2_$TAG 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2_$TAG -o run --output-format csv -- python3 bench.py --steps 200 --no-cpu-baseline --mesh-subdiv 0
  python3 tools/bench_summary.py $OUT/bench_$TAG.log $OUT/bench_c1_$TAG.log $OUT/bench_c3_$TAG.log || true
fi
if [ "$STEPS" = all ] || [ "$STEPS" = shard ]; then
  # rank 0's shard of an N-way landmark split of c2 (per-rank step of the strong-scaling headline)
  for n in 1 2 4 8; do
    run shard${n}_$TAG 300 python3 bench.py --shard-of $n --steps 500 --ba-iters 3 --no-cpu-baseline --mesh-subdiv 0
  done
  python3 tools/bench_summary.py $OUT/shard*_$TAG.log || true
fi
if [ "$STEPS" = ab ]; then
  # same-box A/B against other builds of the ABI (BASE="path/libmvba.so ..." through
  # MVBA_LIB; "cur" = the in-tree library), alternated twice
  for k in 1 2; do
    for v in $BASE cur; do
      if [ $v = cur ]; then unset MVBA_LIB; t=cur; else export MVBA_LIB=$PWD/$v; t=$(basename $(dirname $v)); fi
      for c in ${AB_CFGS:-c2 s8 c3}; do
        case $c in
          c2) run ab_c2_${t}_${k}_$TAG 300 python3 bench.py --steps 2000 --ba-iters 3 --no-cpu-baseline --mesh-subdiv 0 ;;
          s8) run ab_s8_${t}_${k}_$TAG 300 python3 bench.py --shard-of 8 --steps 500 --ba-iters 3 --no-cpu-baseline --mesh-subdiv 0 ;;
          c3) run ab_c3_${t}_${k}_$TAG 400 python3 bench.py --config c3 --steps 30 --ba-iters 2 --no-cpu-baseline --mesh-subdiv 0 ;;
        esac
      done
    done
  done
  unset MVBA_LIB
  python3 tools/bench_summary.py $OUT/ab_*_$TAG.log || true
fi
if [ "$STEPS" = abk ]; then
  # same-box kernel-trace A/B of the CG iteration (BASE as for ab): per-kernel
  # medians over the non-gated iterations (tools/cg_iter_med.py)
  for k in 1 2; do
    for v in $BASE cur; do
      if [ $v = cur ]; then unset MVBA_LIB; t=cur; else export MVBA_LIB=$PWD/$v; t=$(basename $(dirname $v)); fi
      for c in ${AB_CFGS:-c2 s8 c3}; do
        case $c in
          c2) A="--ba-iters 5" ;;
          s8) A="--shard-of 8 --ba-iters 5" ;;
          c3) A="--config c3 --ba-iters 2" ;;
        esac
        run kt_${c}_${t}_${k}_$TAG 400 rocprofv3 --kernel-trace -d $OUT/kt_${c}_${t}_${k}_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --mesh-subdiv 0 $A
        python3 tools/cg_iter_med.py ${c}_${t}_${k} $(find $OUT/kt_${c}_${t}_${k}_$TAG -name '*kernel_trace.csv' | head -1) | tee -a $OUT/cg_iter_$TAG.txt
        find $OUT/kt_${c}_${t}_${k}_$TAG -name '*kernel_trace.csv' -exec gzip {} \;
      done
    done
  done
  unset MVBA_LIB
fi
if [ "$STEPS" = configs ]; then
  # the BASELINE.md table's other rows: c4 whole on one GPU, c5 (depth, fp32 eval line)
  run bench_c5_$TAG 600 python3 bench.py --config c5 --steps 200 --mesh-subdiv 0 --cpu-sample 1000000
  run bench_c4_$TAG 900 python3 bench.py --config c4 --steps 20 --ba-iters 2 --mesh-subdiv 0 --cpu-sample 1000000
  python3 tools/bench_summary.py $OUT/bench_c5_$TAG.log $OUT/bench_c4_$TAG.log || true
fi
if [ "$STEPS" = chol ]; then
  # X1 pricing: hand-written fp64-MFMA blocked Cholesky vs rocSOLVER dpotrf (tools/chol_bench.hip)
  run chol512_$TAG 120 tools/chol_bench 512
  run chol_$TAG 400 tools/chol_bench 21248
fi
if [ "$STEPS" = pmc ]; then
  # per-launch HBM traffic of the evaluation launch (k_eval_local, the default form) and of K1 (k_obs), separate FETCH / WRITE passes
  for CFG in ${PMC_CFGS:-c2 c3}; do
    B="python3 bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline --ba-iters 0 --mesh-subdiv 0"
    run fetch_${CFG}_$TAG 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_${CFG}_$TAG -o run --output-format csv -- $B
    run write_${CFG}_$TAG 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write_${CFG}_$TAG -o run --output-format csv -- $B
    D=$(python3 -c "import sys; sys.path.insert(0, '.'); from multiview_amd import rig; from bench import kernel_degree; m = rig.CONFIGS['$CFG']['models'][0]; print(kernel_degree(m))")
    python3 tools/pmc_summary.py $OUT/fetch_${CFG}_$TAG/run_counter_collection.csv $OUT/write_${CFG}_$TAG/run_counter_collection.csv "k_eval_local<$D, double, true>" $OUT/pmc_eval_${CFG}.json $CFG
    python3 tools/pmc_summary.py $OUT/fetch_${CFG}_$TAG/run_counter_collection.csv $OUT/write_${CFG}_$TAG/run_counter_collection.csv "k_obs<$D, double>" $OUT/pmc_k1_${CFG}.json $CFG
  done
fi
if [ "$STEPS" = tests ] && [ -n "${TESTS:-}" ]; then :; fi
exit 0
