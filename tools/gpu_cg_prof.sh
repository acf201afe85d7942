#!/bin/bash
# CG-iteration anatomy: rocprof kernel trace of the c2 BA phase (phase C only
# matters; the other phases are short), then tools/cg_period.py on it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
CFG=${1:-c2}
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_cg -o run --output-format csv -- \
  python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof_cg.log 2>&1 || exit $?
f=$(find $OUT/prof_cg -name '*kernel_trace.csv' | head -1)
python3 tools/cg_period.py "$f" | tee $OUT/cg_period_$CFG.txt
