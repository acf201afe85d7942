#!/bin/bash
# GPU session: parity tests + store-pattern ceilings + PMC traffic of the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-r01b}
run() {
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc" | tee -a $OUT/steps.log
  tail -12 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider
run store_bench 120 ./tools/store_bench 1000000 56
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch_$TAG -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write_$TAG -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
exit 0
