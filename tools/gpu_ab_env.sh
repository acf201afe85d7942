#!/bin/bash
# Same-box A/B of an environment switch: tools/gpu_ab_env.sh VAR [config]
# runs tools/solve_probe.py under rocprofv3 with VAR=0,1,0,1 and prints the
# per-kernel average of each run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
var=$1; cfg=${2:-c2}
mkdir -p gpurun_out/ab_env
for k in 1 2; do for v in 0 1; do
  export $var=$v
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_env/${var}_${v}_$k -o run --output-format csv -- python3 tools/solve_probe.py --config $cfg > gpurun_out/ab_env/${var}_${v}_$k.log 2>&1 || { tail -5 gpurun_out/ab_env/${var}_${v}_$k.log; exit 1; }
  echo "$var=$v run $k: $(grep LM gpurun_out/ab_env/${var}_${v}_$k.log)"
  f=$(find gpurun_out/ab_env/${var}_${v}_$k -name run_kernel_stats.csv | head -1)
  python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:8]:
    print(f"   {r['Name'][:60]:60s} {r['Calls']:>6s} {float(r['AverageNs'])/1000:8.1f}")
PY
done; done
