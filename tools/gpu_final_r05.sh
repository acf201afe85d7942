#!/bin/bash
# Round-5 final-tree evidence: GPU tests + smoke, the default bench line (c2 with
# the CPU baseline), c1 / c3 / c5 / c4 lines, rocprofv3 kernel stats of the c2
# bench (its k_eval_local average against the line's roofline.kernel_ms), the
# shard rehearsal (rank 0's 1/N shard of c2 at N = 1, 2, 4, 8), rocm-smi clocks.
# Steps chained: the script stops at the first fault / abort / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-r05z}
STEPS=${2:-all}
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps_$TAG.log
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc" | tee -a $OUT/steps_$TAG.log
  tail -3 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
rocm-smi --showclocks --showpower --showmaxpower --showtemp --showmeminfo vram > $OUT/smi_$TAG.txt 2>&1 || true
if [ "$STEPS" = all ] || [ "$STEPS" = tests ]; then
  run pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread
  run smoke_$TAG 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$STEPS" = all ] || [ "$STEPS" = bench ]; then
  run bench_$TAG 600 python bench.py
  run bench_c1_$TAG 300 python bench.py --config c1 --mesh-subdiv 0
  run bench_c3_$TAG 600 python bench.py --config c3 --steps 50 --mesh-subdiv 0 --cpu-sample 200000
  run bench_c5_$TAG 600 python bench.py --config c5 --steps 200 --mesh-subdiv 0 --cpu-sample 1000000
  run prof_c2_$TAG 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2_$TAG -o run --output-format csv -- python3 bench.py --steps 200 --no-cpu-baseline --mesh-subdiv 0
  python3 tools/bench_summary.py $OUT/bench_$TAG.log $OUT/bench_c1_$TAG.log $OUT/bench_c3_$TAG.log $OUT/bench_c5_$TAG.log || true
fi
if [ "$STEPS" = all ] || [ "$STEPS" = shard ]; then
  for n in 1 2 4 8; do
    run shard${n}_$TAG 300 python3 bench.py --shard-of $n --steps 500 --ba-iters 5 --no-cpu-baseline --mesh-subdiv 0
  done
  python3 tools/bench_summary.py $OUT/shard*_$TAG.log || true
fi
if [ "$STEPS" = all ] || [ "$STEPS" = c4 ]; then
  run bench_c4_$TAG 900 python3 bench.py --config c4 --steps 20 --ba-iters 2 --mesh-subdiv 0 --cpu-sample 1000000
fi
exit 0
