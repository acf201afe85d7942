#!/bin/bash
# Round-2 evidence refresh: smoke, default bench under rocprofv3 kernel stats,
# c3 and c5 bench lines. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ev
mkdir -p $OUT
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step prof_c2 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o run --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline --mesh-subdiv 0
step bench_c3 600 python3 bench.py --config c3 --no-cpu-baseline --mesh-subdiv 0
step bench_c5 600 python3 bench.py --config c5 --no-cpu-baseline --mesh-subdiv 0
for f in prof_c2 bench_c3 bench_c5; do python3 tools/bench_summary.py $OUT/$f.log; done
exit 0
