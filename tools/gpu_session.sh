#!/bin/bash
# One parameterised GPU lease script (replaces the per-session tools/gpu_r0*.sh).
#
#   tools/gpu_session.sh TAG STEP[,STEP...]
#
# Steps (run in the order given; outputs under gpurun_out/, named *_TAG):
#   tests      pytest -m gpu (TESTS=... narrows it, PYTEST_ARGS adds options)
#   smoke      __graft_entry__.smoke()
#   bench      the default bench line (c2, CPU baseline) + c1 and c3 lines
#   bench45    the c4 (50M observations) and c5 (depth) bench lines
#   prof       rocprofv3 --kernel-trace --stats of the c2 bench (roofline.kernel_ms check)
#   shard      rank 0's shard of an N-way landmark split of c2, N = 1 2 4 8
#              (bench.py --shard-of N): the per-rank step of the strong-scaling headline
#   rccl       the same shards' LM phase through a one-rank RCCL communicator
#              (bench.py --ba-exchange rccl: the sharded solve's code path, graphs
#              with the exchange inside), with MVBA_CG_TIMING=1's host/GPU split
#   kt         kernel traces of the CG iteration (tools/gpu_kt.sh; KT_CFGS, KT_VARS)
#   ab         same-box A/B of bench lines against other builds (BASE="tools/ab/X/libmvba.so ...",
#              AB_CFGS="c2 s8 c3"); the in-tree library is "cur"
#   envab      same-box A/B of bench lines under env variants, with MVBA_CG_TIMING=1
#              (ENV_VARS="name=VAR=V,VAR=V name2=..." ; ENV_CFGS="s8 r8 c2"), twice each
#   pmc        PMC passes per config (tools/gpu_pmc.sh; PMC_CFGS)
#   baroof     BA roofline of one CG iteration (tools/gpu_ba_roofline.sh; BA_CFGS)
#
# Every GPU step has its own time limit; the script stops at the first fault,
# abort, segfault, timeout or hang (exit codes other than 0 and pytest's 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:?usage: gpu_session.sh TAG STEP[,STEP...]}
STEPS=${2:-tests,smoke,bench}
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
NB="--no-cpu-baseline --mesh-subdiv 0"
for step in ${STEPS//,/ }; do
  case $step in
    tests)
      run pytest_gpu_$TAG ${TESTS_SECS:-900} python -u -m pytest ${TESTS:-tests} -m gpu -q -p no:cacheprovider \
        --timeout 400 --timeout-method thread ${PYTEST_ARGS:-} ;;
    smoke)
      run smoke_$TAG 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      run bench_$TAG 600 python bench.py
      run bench_c1_$TAG 300 python bench.py --config c1 --mesh-subdiv 0
      run bench_c3_$TAG 600 python bench.py --config c3 --steps 50 --mesh-subdiv 0 --cpu-sample 200000
      python3 tools/bench_summary.py $OUT/bench_$TAG.log $OUT/bench_c1_$TAG.log $OUT/bench_c3_$TAG.log || true ;;
    bench45)
      run bench_c4_$TAG 400 python3 bench.py --config c4 --steps 20 --ba-iters 2 --mesh-subdiv 0 --cpu-sample 1000000
      run bench_c5_$TAG 400 python3 bench.py --config c5 --mesh-subdiv 0
      python3 tools/bench_summary.py $OUT/bench_c4_$TAG.log $OUT/bench_c5_$TAG.log || true ;;
    prof)
      run prof_c2_$TAG 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2_$TAG -o run --output-format csv -- \
        python3 bench.py --steps 200 $NB ;;
    shard)
      for n in 1 2 4 8; do
        run shard${n}_$TAG 300 python3 bench.py --shard-of $n --steps 500 --ba-iters ${SHARD_BA_ITERS:-3} $NB
      done
      python3 tools/bench_summary.py $OUT/shard*_$TAG.log || true ;;
    rccl)
      for n in ${RCCL_SHARDS:-1 8}; do
        MVBA_CG_TIMING=1 run rccl${n}_$TAG 300 python3 bench.py --shard-of $n --ba-exchange rccl --steps 200 \
          --ba-iters ${SHARD_BA_ITERS:-5} $NB
        grep -h "cg timing\|graph capture" $OUT/rccl${n}_$TAG.log || true
      done
      python3 tools/bench_summary.py $OUT/rccl*_$TAG.log || true ;;
    kt)
      REPS=${REPS:-1} bash tools/gpu_kt.sh $TAG "${KT_CFGS:-s8 c2}" "${KT_VARS:-cur=MVBA_CG_GRAPH=1}" || exit 1 ;;
    ab)
      for k in 1 2; do
        for v in ${BASE:-} cur; do
          if [ $v = cur ]; then unset MVBA_LIB; t=cur; else export MVBA_LIB=$PWD/$v; t=$(basename $(dirname $v)); fi
          for c in ${AB_CFGS:-c2 s8 c3}; do
            case $c in
              c2) run ab_c2_${t}_${k}_$TAG 300 python3 bench.py --steps 2000 --ba-iters 3 $NB ;;
              s8) run ab_s8_${t}_${k}_$TAG 300 python3 bench.py --shard-of 8 --steps 500 --ba-iters 3 $NB ;;
              r8) run ab_r8_${t}_${k}_$TAG 300 python3 bench.py --shard-of 8 --ba-exchange rccl --steps 200 --ba-iters 5 $NB ;;
              c3) run ab_c3_${t}_${k}_$TAG 400 python3 bench.py --config c3 --steps 30 --ba-iters 2 $NB ;;
            esac
          done
        done
      done
      unset MVBA_LIB
      python3 tools/bench_summary.py $OUT/ab_*_$TAG.log || true ;;
    envab)
      for k in 1 2; do
        for v in ${ENV_VARS:-cur=MVBA_CG_GRAPH=1}; do
          name=${v%%=*}; envs=${v#*=}
          for c in ${ENV_CFGS:-s8 r8 c2}; do
            case $c in
              c2) A="--steps 500 --ba-iters 5" ;;
              s8) A="--shard-of 8 --steps 200 --ba-iters 5" ;;
              r8) A="--shard-of 8 --ba-exchange rccl --steps 200 --ba-iters 5" ;;
              c3) A="--config c3 --steps 30 --ba-iters 2" ;;
            esac
            env ${envs//,/ } MVBA_CG_TIMING=1 timeout -k 10 300 python3 bench.py $A $NB > $OUT/envab_${c}_${name}_${k}_$TAG.log 2>&1
            rc=$?
            if [ $rc -ne 0 ]; then echo "envab $c $name failed (rc=$rc)"; tail -3 $OUT/envab_${c}_${name}_${k}_$TAG.log; exit $rc; fi
            echo "$c $name $k: $(grep 'cg timing' $OUT/envab_${c}_${name}_${k}_$TAG.log | sed -n 2p | sed 's/.*| us per solve/us per solve/')"
          done
        done
      done
      python3 tools/bench_summary.py $OUT/envab_*_$TAG.log || true ;;
    pmc)
      PMC_CFGS=${PMC_CFGS:-c2} bash tools/gpu_pmc.sh $TAG || exit 1 ;;
    baroof)
      for c in ${BA_CFGS:-c2}; do bash tools/gpu_ba_roofline.sh $c $TAG || exit 1; done ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
