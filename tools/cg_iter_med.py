#!/usr/bin/env python3
"""Median CG iteration (pass A -> update span, or the fused step's period,
boundaries included) and the median of each of its kernels over the non-gated
iterations of a rocprofv3 kernel trace (tools/ba_roofline.py's selection).
usage: cg_iter_med.py LABEL run_kernel_trace.csv [...]"""
import statistics as st
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from ba_roofline import trace_iterations  # noqa: E402

args = sys.argv[1:]
for label, path in zip(args[0::2], args[1::2]):
    its, seq = trace_iterations(path)
    if not its:
        print(f"{label:24s} no non-gated CG iterations")
        continue
    parts = "  ".join(f"{k.replace('k_', '')} {st.median(i[k] for i in its):6.2f}" for k in seq)
    print(f"{label:24s} n={len(its):4d} span {st.median(i['span_us'] for i in its):7.2f} us | {parts}")
