#!/usr/bin/env python3
"""Median duration per kernel over its launches longer than a gate threshold
(CG launches past the stop return at once: ~2-5 us), from a rocprofv3 kernel
trace. usage: ktrace_med.py run_kernel_trace.csv [min_us=8]"""
import csv
import re
import statistics as st
import sys
from collections import defaultdict

path = sys.argv[1]
lo = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
d = defaultdict(list)
for r in csv.DictReader(open(path)):
    k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("mvba::", "")
    d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k in ("k_pass_a_frame", "k_point_w", "k_pass_b", "k_vec_rep_reduce", "k_cg_update", "k_frame_lin", "k_eval", "k_obs<",
          "k_block_prec", "k_pass_a<", "k_pass_sq"):
    for name, v in d.items():
        if name.startswith(k):
            w = [x for x in v if x >= lo]
            if w:
                print(f"{name[:36]:36s} n={len(w):4d} median {st.median(w):9.2f} us")
