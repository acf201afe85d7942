#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counter CSVs (one pass per CSV).

usage: pmc_solver.py OUT.json run_counter_collection.csv [more.csv ...]

Every dispatch contributes one row per counter; this averages each counter over
the dispatches of each kernel (gated CG launches included, which is why the
launch count is printed beside it) and derives, where the counters are present:
  fetch_MB        FETCH_SIZE (KB) x 2 / 1e3: gfx950 tallies 128-B requests at 64 B
                  (MI355X_MICROARCH.md, HBM section) -> corrected MB per launch
  write_MB        WRITE_SIZE (KB) / 1e3
  wait_frac       SQ_WAIT_ANY / SQ_WAVE_CYCLES          (waves parked on s_waitcnt)
  inst_wait_frac  SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES     (issue stalls)
  active_frac     SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  valu_busy       SQ_ACTIVE_INST_VALU / (SQ_BUSY_CYCLES * 4 SIMDs * CUs per SE)
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "").replace("mvba::", "")
    return name.strip()


def load(path, acc, calls):
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            c = r["Counter_Name"]
            acc[k][c] += float(r["Counter_Value"])
            calls[k][c] += 1
            dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            acc[k]["_dur_ns_" + c] += dur


def main():
    out = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(lambda: defaultdict(int))
    for p in sys.argv[2:]:
        load(p, acc, calls)
    res = {}
    for k, cs in acc.items():
        row = {}
        for c, v in cs.items():
            if c.startswith("_dur_ns_"):
                continue
            n = calls[k][c]
            row[c] = v / n
            row["launches_" + c] = n
        if "FETCH_SIZE" in row:
            row["fetch_MB"] = row["FETCH_SIZE"] * 2 / 1e3
        if "WRITE_SIZE" in row:
            row["write_MB"] = row["WRITE_SIZE"] / 1e3
        wc = row.get("SQ_WAVE_CYCLES")
        if wc:
            for c, nm in (("SQ_WAIT_ANY", "wait_frac"), ("SQ_WAIT_INST_ANY", "inst_wait_frac"),
                          ("SQ_ACTIVE_INST_ANY", "active_frac")):
                if c in row:
                    row[nm] = row[c] / wc
        res[k] = row
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    keys = ("launches_FETCH_SIZE", "fetch_MB", "write_MB", "wait_frac", "inst_wait_frac", "active_frac",
            "SQ_INSTS_VALU", "SQ_WAVES")
    print("kernel".ljust(44), " ".join(s[:14].rjust(14) for s in keys))
    for k in sorted(res, key=lambda k: -res[k].get("fetch_MB", 0.0)):
        print(k[:44].ljust(44), " ".join(
            ("%14.3f" % res[k][s]) if s in res[k] else " " * 14 for s in keys))


if __name__ == "__main__":
    main()
