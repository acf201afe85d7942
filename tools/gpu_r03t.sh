#!/bin/bash
# Sharded CG tail folded into the replica reduction (rank 0 adds the damping
# before the exchange, the update kernel takes the step from the exchanged
# p.q): solver / sharded GPU tests, then the 2-shard local-communicator
# rehearsal with the fold on and off (MVBA_CG_FOLD=0), alternated twice; then
# c5 and rank 0's shard of the 8-way c4 split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03t}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_solver_gpu.py tests/test_deterministic_gpu.py tests/test_depth.py tests/test_cli.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_fold_$TAG.log 2>&1
rc=$?; tail -2 $OUT/pytest_fold_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_fold_$TAG.log | head; exit $rc; }
for k in 1 2; do
  for v in 1 0; do
    f=$OUT/shardreh_fold${v}_${k}_$TAG.log
    timeout -k 10 300 env MVBA_CG_FOLD=$v python3 tools/shard_rehearsal.py --config c2 --shards 2 --iters 5 > $f 2>&1 || { tail -3 $f; exit 1; }
    echo "fold=$v: $(grep '^{' $f | head -1 | cut -c1-400)"
  done
done
timeout -k 10 400 python3 bench.py --config c5 --steps 10 --no-cpu-baseline > $OUT/bench_c5_$TAG.log 2>&1 || { tail -5 $OUT/bench_c5_$TAG.log; exit 1; }
python3 tools/bench_summary.py $OUT/bench_c5_$TAG.log
timeout -k 10 500 python3 bench.py --config c4 --shard-of 8 --steps 5 --ba-iters 3 --no-cpu-baseline > $OUT/bench_c4_shard8_$TAG.log 2>&1 || { tail -5 $OUT/bench_c4_shard8_$TAG.log; exit 1; }
python3 tools/bench_summary.py $OUT/bench_c4_shard8_$TAG.log
exit 0
