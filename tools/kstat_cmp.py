"""Compare per-kernel average durations of two rocprofv3 kernel_stats.csv files.

usage: python tools/kstat_cmp.py A/run_kernel_stats.csv B/run_kernel_stats.csv [n]
"""
import csv
import sys


def load(path):
    out = {}
    for r in csv.DictReader(open(path)):
        name = r["Name"]
        name = name.split("(")[0] if not name.startswith("void ") else name[5:].split("(")[0]
        out[name] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e3)
    return out


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    names = sorted(set(a) | set(b), key=lambda k: -max(a.get(k, (0, 0, 0))[2], b.get(k, (0, 0, 0))[2]))
    print(f"{'kernel':48s} {'calls A':>7s} {'avg A us':>9s} {'calls B':>7s} {'avg B us':>9s}")
    for k in names[:n]:
        ca, ta, _ = a.get(k, (0, float("nan"), 0))
        cb, tb, _ = b.get(k, (0, float("nan"), 0))
        print(f"{k[:48]:48s} {ca:7d} {ta:9.1f} {cb:7d} {tb:9.1f}")


if __name__ == "__main__":
    main()
