#!/bin/bash
# Round-4 evidence session: GPU tests, smoke, the default bench line (c2, CPU
# baseline), c1 and c3 lines, and a rocprofv3 kernel-trace summary of the c2
# bench whose k_eval average the line's roofline.kernel_ms must match.
# Each GPU step has its own time limit; the script stops at the first fault,
# abort, segfault, timeout or hang (exit codes other than 0 and pytest's 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-r04}
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
  run pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread
  run smoke_$TAG 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$STEPS" = all ] || [ "$STEPS" = bench ]; then
  run bench_$TAG 600 python bench.py
  run bench_c1_$TAG 300 python bench.py --config c1 --mesh-subdiv 0
  run bench_c3_$TAG 600 python bench.py --config c3 --steps 50 --no-cpu-baseline --mesh-subdiv 0
  run prof_c2_$TAG 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2_$TAG -o run --output-format csv -- python3 bench.py --steps 200 --no-cpu-baseline --mesh-subdiv 0
  python3 tools/bench_summary.py $OUT/bench_$TAG.log $OUT/bench_c1_$TAG.log $OUT/bench_c3_$TAG.log || true
fi
if [ "$STEPS" = all ] || [ "$STEPS" = shard ]; then
  # slot alignment 32 (default) vs 16 on the whole c2 and on rank 0's 1/8 shard, alternated
  for k in 1 2; do
    for a in 32 16; do
      for n in 1 8; do
        run shard${n}_a${a}_${k}_$TAG 300 env MVBA_SLOT_ALIGN=$a python3 bench.py --shard-of $n --steps 500 --ba-iters 3 --no-cpu-baseline --mesh-subdiv 0
      done
    done
  done
  python3 tools/bench_summary.py $OUT/shard*_$TAG.log || true
fi
exit 0
