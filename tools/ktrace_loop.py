#!/usr/bin/env python3
"""The timed loop's launches of one kernel in a rocprofv3 kernel trace: the
longest run of consecutive dispatches of that kernel (bench.py's K back-to-back
steps), their mean / median duration and their start-to-start period, as a
JSON summary to set beside the bench line's roofline.kernel_ms.

    ktrace_loop.py run_kernel_trace.csv 'k_eval<2, 0, double, true>' [out.json]
"""
import csv
import json
import statistics as st
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    best, cur = [], []
    for r in rows:
        if name in r["Kernel_Name"]:
            cur.append(r)
            if len(cur) > len(best):
                best = list(cur)
        else:
            cur = []
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in best]
    per = [(int(b["Start_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3 for a, b in zip(best, best[1:])]
    allv = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if name in r["Kernel_Name"]]
    out = {"kernel": name, "trace": path, "loop_launches": len(best),
           "loop_mean_us": st.mean(dur), "loop_median_us": st.median(dur),
           "loop_period_us": st.mean(per) if per else None,
           "all_launches": len(allv), "all_mean_us": st.mean(allv)}
    print(json.dumps(out))
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
