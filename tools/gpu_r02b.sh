#!/bin/bash
# round 2 session b: solver + full-size tests, shard rehearsal, bench, gloo 2-rank rehearsal
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/pytest_gpu_r02b.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu_r02b.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/shard_rehearsal.py --config c2 --shards 2 --iters 5 > gpurun_out/shard_rehearsal_r02b.log 2>&1 || { tail -20 gpurun_out/shard_rehearsal_r02b.log; exit 3; }
tail -2 gpurun_out/shard_rehearsal_r02b.log
timeout -k 10 300 python bench.py > gpurun_out/bench_r02b.log 2>&1 || { tail -20 gpurun_out/bench_r02b.log; exit 4; }
tail -c 1500 gpurun_out/bench_r02b.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline > gpurun_out/bench_gloo2_r02b.log 2>&1
echo gloo2 rc $?
tail -c 2500 gpurun_out/bench_gloo2_r02b.log
