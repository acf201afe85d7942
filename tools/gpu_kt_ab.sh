#!/bin/bash
# Same-box kernel-trace A/B of environment switches over the CG iteration:
#   tools/gpu_kt_ab.sh TAG "c3 c2 s8" LABEL:VAR=VAL,VAR=VAL LABEL2: ...
# (a variant with nothing after the colon runs the defaults; config s8 = rank
# 0's shard of an 8-way c2 split), each run twice, then tools/cg_iter_med.py over
# every trace into gpurun_out/kt_TAG/cg_iter.txt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; CFGS=$2; shift 2
OUT=gpurun_out/kt_$TAG
mkdir -p $OUT
args=()
for rep in 1 2; do
  for cfg in $CFGS; do
    for var in "$@"; do
      label=${var%%:*}; envs=${var#*:}
      case $cfg in
        s8) extra="--shard-of 8 --ba-iters 5";;
        c3) extra="--config c3 --ba-iters 2";;
        *) extra="--config $cfg --ba-iters 5";;
      esac
      name=${cfg}_${label}_$rep
      ( IFS=,; for kv in $envs; do export "$kv"; done; unset IFS
        timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/$name -o run --output-format csv -- \
          python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --mesh-subdiv 0 $extra > $OUT/$name.log 2>&1 ) \
        || { echo "$name failed"; tail -5 $OUT/$name.log; exit 1; }
      f=$(find $OUT/$name -name '*kernel_trace.csv' | head -1)
      args+=("$name" "$f")
      echo "$name: $(python3 tools/bench_summary.py $OUT/$name.log)"
    done
  done
done
python3 tools/cg_iter_med.py "${args[@]}" | tee $OUT/cg_iter.txt
for a in "${args[@]}"; do case $a in *.csv) gzip -f "$a";; esac; done
