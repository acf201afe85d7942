#!/bin/bash
# Solver iteration: GPU solver tests, then rocprof kernel stats of the c2 bench
# (all phases) -> gpurun_out/prof_solver/ and a short summary; CONFIGS="c2 c3"
# profiles more workloads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_solver_gpu.py tests/test_xyz_prior.py tests/test_depth.py -x -q -m gpu \
  > $OUT/solver_tests.log 2>&1
rc=$?
tail -2 $OUT/solver_tests.log
[ $rc -ne 0 ] && exit $rc
for cfg in ${CONFIGS:-c2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_solver_$cfg -o run --output-format csv -- \
    python3 bench.py --config $cfg --steps 10 --no-cpu-baseline > $OUT/prof_solver_$cfg.log 2>&1
  rc=$?
  [ $rc -ne 0 ] && { tail -5 $OUT/prof_solver_$cfg.log; exit $rc; }
  grep -o '"ba": {[^}]*}' $OUT/prof_solver_$cfg.log | cut -c1-400
  CFG=$cfg python3 - <<'PY'
import csv, glob, os
f = glob.glob(f"gpurun_out/prof_solver_{os.environ['CFG']}/**/*kernel_stats.csv", recursive=True)
if f:
    r = list(csv.DictReader(open(f[0])))
    for x in r[:12]:
        print(x["Name"][:48].ljust(48), x["Calls"].rjust(6), "%9.1f us" % (float(x["AverageNs"]) / 1e3))
PY
done
exit 0
