#!/bin/bash
# GPU session producing the round's evidence: GPU tests, default bench (with the
# CPU baseline), c3 / c5 bench lines, rocprof kernel stats for c2 and c5, two
# PMC passes (FETCH_SIZE, WRITE_SIZE: they cannot share a pass on gfx950) for
# K1's HBM traffic (summarised into pmc_k1_c2.json), and an MFMA pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-r01}
run() {
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
K1='k_obs<2, 0, double>'
run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider
run bench_$TAG 600 python bench.py
run bench_c3_$TAG 600 python bench.py --config c3 --steps 10 --no-cpu-baseline
run bench_c5_$TAG 600 python bench.py --config c5 --no-cpu-baseline
run prof_c2_$TAG 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2_$TAG -o run --output-format csv -- python3 bench.py --steps 10 --no-cpu-baseline
run prof_c5_$TAG 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5_$TAG -o run --output-format csv -- python3 bench.py --config c5 --steps 10 --no-cpu-baseline
run pmc_fetch_$TAG 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --ba-iters 0
run pmc_write_$TAG 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --ba-iters 0
python3 tools/pmc_summary.py $OUT/pmc_fetch_$TAG/run_counter_collection.csv $OUT/pmc_write_$TAG/run_counter_collection.csv "$K1" $OUT/pmc_k1_c2.json c2
# MFMA use of the K2 Gram kernels (fp64 v_mfma_f64_16x16x4f64): busy cycles vs wall
run pmc_mfma_$TAG 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $OUT/pmc_mfma_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --ba-iters 2
python3 tools/bench_summary.py $OUT/bench_$TAG.log $OUT/bench_c3_$TAG.log $OUT/bench_c5_$TAG.log
exit 0
