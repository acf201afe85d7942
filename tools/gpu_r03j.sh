#!/bin/bash
# Kernel-level A/B (rocprofv3 kernel traces) of base / pass-A pipe 1 / pipe 2
# at c2 and c3; tools/ktrace_med.py prints per-kernel medians of non-gated launches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for cfg in c2 c3; do
  for v in base pipe1 pipe2; do
    case $v in
      base) export MVBA_LIB=tools/ab/base/libmvba.so; unset MVBA_PASS_A_PIPE ;;
      pipe1) unset MVBA_LIB; export MVBA_PASS_A_PIPE=1 ;;
      pipe2) unset MVBA_LIB; export MVBA_PASS_A_PIPE=2 ;;
    esac
    if [ $cfg = c3 ]; then A="--config c3 --steps 3 --ba-iters 3"; else A="--steps 5 --ba-iters 5"; fi
    timeout -s KILL 240 rocprofv3 --kernel-trace -d $OUT/kt_${cfg}_$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --mesh-subdiv 0 $A > $OUT/kt_${cfg}_$v.log 2>&1 || { tail -3 $OUT/kt_${cfg}_$v.log; exit 1; }
    echo "== $cfg $v"; python3 tools/ktrace_med.py $OUT/kt_${cfg}_$v/run_kernel_trace.csv
  done
done
exit 0
