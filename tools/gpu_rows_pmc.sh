#!/bin/bash
# PMC passes over k_rows (tools/rows_probe.py), one counter group per run
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/rows_pmc
timeout -k 10 120 python3 tools/rows_probe.py > gpurun_out/rows_pmc/plain.log 2>&1 || exit 1
tail -3 gpurun_out/rows_pmc/plain.log
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex k_rows -d gpurun_out/rows_pmc/p$i -o run --output-format csv -- python3 tools/rows_probe.py > gpurun_out/rows_pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/rows_pmc/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/rows_pmc/p*/**/run_counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    # per dispatch totals: counters are per dimension instance; sum per dispatch would need grouping
    print(f, {k: sum(v) / 6 for k, v in acc.items()})
PY
