"""Per-kernel median duration over the non-gated launches (> 4 us) of two
rocprofv3 kernel traces (gated CG iterations past the stop return at once and
would dilute a plain average).

usage: python tools/ktrace_cmp.py A/run_kernel_trace.csv B/run_kernel_trace.csv [n]
"""
import csv
import statistics
import sys
from collections import defaultdict


def load(path):
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        name = name[5:] if name.startswith("void ") else name
        d[name.split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return d


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    keys = sorted(set(a) | set(b), key=lambda k: -max(sum(a.get(k, [0])), sum(b.get(k, [0]))))
    print(f"{'kernel':44s} {'n A':>5s} {'med A':>7s} {'n B':>5s} {'med B':>7s}")
    for k in keys[:n]:
        la = [t for t in a.get(k, []) if t > 4.0] or [float("nan")]
        lb = [t for t in b.get(k, []) if t > 4.0] or [float("nan")]
        print(f"{k[:44]:44s} {len(la):5d} {statistics.median(la):7.1f} {len(lb):5d} {statistics.median(lb):7.1f}")


if __name__ == "__main__":
    main()
