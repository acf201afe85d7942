#!/bin/bash
# Kernel trace of rank 0's shard of an 8-way c2 split (BA phase): where a thin
# shard's CG iteration goes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
d=$OUT/kt_shard8_r03i2
timeout -s KILL 300 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 bench.py --shard-of 8 --steps 5 --ba-iters 5 --no-cpu-baseline --mesh-subdiv 0 > $d.log 2>&1 || { tail -3 $d.log; exit 1; }
python3 tools/bench_summary.py $d.log
python3 tools/ktrace_med.py $d/run_kernel_trace.csv 0

exit 0
