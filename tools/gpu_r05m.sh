#!/bin/bash
# c3 across trees on one box (tools/gpu_r05l.sh's A/B), then the final-tree evidence
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r05m}
for k in 1 2; do
  for v in r04x cur; do
    if [ $v = cur ]; then unset MVBA_LIB; else export MVBA_LIB=$PWD/tools/ab/$v/libmvba.so; fi
    timeout -k 10 400 python bench.py --config c3 --steps 400 --no-cpu-baseline --mesh-subdiv 0 --ba-iters 0 > $OUT/c3eval_${v}_${k}_$TAG.log 2>&1 &
    pid=$!
    sleep 45
    rocm-smi --showclocks --showpower --showtemp > $OUT/smi_c3eval_${v}_${k}_$TAG.txt 2>&1
    wait $pid || { echo "bench failed ($v $k)"; exit 1; }
    echo "$v $k: $(python3 tools/bench_summary.py $OUT/c3eval_${v}_${k}_$TAG.log | tail -1 | cut -c1-110) | $(grep -E 'sclk|mclk|Power' $OUT/smi_c3eval_${v}_${k}_$TAG.txt | tr -s ' \t' ' ' | tr '\n' ';')"
  done
done
unset MVBA_LIB
bash tools/gpu_final_r05.sh $TAG
