#!/bin/bash
# kernel traces of the CG iteration (median span + per-kernel medians over the
# non-gated iterations, tools/cg_iter_med.py) for the listed configs and env
# variants: usage gpu_kt.sh TAG "cfg ..." "NAME=ENV,ENV NAME=ENV ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-kt}
CFGS=${2:-"s8 c2"}
VARS=${3:-"cur=MVBA_CG_GRAPH=1"}
for k in ${REPS:-1}; do
for cfg in $CFGS; do
  case $cfg in s8) A="--shard-of 8 --ba-iters 5";; c2) A="--ba-iters 5";; c3) A="--config c3 --ba-iters 2";;
    r8) A="--shard-of 8 --ba-exchange rccl --ba-iters 5";; esac
  for v in $VARS; do
    name=${v%%=*}; envs=${v#*=}
    D=$OUT/kt_$TAG/${cfg}_${name}_$k
    env ${envs//,/ } timeout -k 10 400 rocprofv3 --kernel-trace -d $D -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --mesh-subdiv 0 $A > $OUT/kt_${cfg}_${name}_${k}_$TAG.log 2>&1 || { echo "failed $cfg $name"; tail -3 $OUT/kt_${cfg}_${name}_${k}_$TAG.log; exit 1; }
    f=$(find $D -name '*kernel_trace.csv' | head -1)
    python3 tools/cg_iter_med.py ${cfg}_${name}_$k $f | tee -a $OUT/cg_iter_$TAG.txt
    gzip $f
  done
done
done
