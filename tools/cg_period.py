"""CG-iteration anatomy from a rocprofv3 kernel trace: the period between
successive k_pass_a launches of the solve, the busy time of each kernel in it and
the idle gaps between them. Usage: python tools/cg_period.py <kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mvba::", ""), int(r["Start_Timestamp"]),
           int(r["End_Timestamp"])) for r in rows]
    starts = [i for i, k in enumerate(ks) if k[0].startswith("k_pass_a")]
    # keep iterations whose next pass A follows within the same CG run (period < 1 ms)
    per, busy, gap = [], defaultdict(list), []
    for a, b in zip(starts, starts[1:]):
        T = ks[b][1] - ks[a][1]
        if T > 1_000_000:
            continue
        seq = ks[a:b]
        if not any(k[0].startswith("k_pass_b") for k in seq):
            continue
        per.append(T)
        g = 0
        for (n, s, e), nxt in zip(seq, ks[a + 1:b + 1]):
            busy[n].append(e - s)
            g += max(0, nxt[1] - e)
        gap.append(g)
    if not per:
        print("no CG iterations found")
        return
    m = lambda v: sum(v) / len(v) / 1e3
    print(f"iterations {len(per)}  period {m(per):.1f} us  idle gaps {m(gap):.1f} us")
    for n, v in sorted(busy.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {n[:60]:60s} {len(v):5d} x {m(v):7.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
