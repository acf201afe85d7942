#!/bin/bash
# rocprofv3 kernel trace + stats of the c2 bench (tag = $1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-prof}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py --steps 10 --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 || { tail -20 gpurun_out/bench_$tag.log; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_$tag.log
f=$(find gpurun_out/prof_$tag -name "run_kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:28]:
    print(f"{r['Name'][:70]:70s} {r['Calls']:>6s} {float(r['AverageNs'])/1000:8.1f} {float(r['TotalDurationNs'])/1e6:8.2f}")
PY
