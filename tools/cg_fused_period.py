#!/usr/bin/env python3
"""Median CG-iteration period (anchor launch to the next anchor launch, gaps
included) over working iterations of a rocprofv3 kernel trace, for both CG
forms: the anchor is pass A (k_pass_a_frame) or the fused step (k_upd_pass_a,
the update of iteration i-1 inside pass A of iteration i). Iterations whose
launches between the two anchors are not exactly one CG product (residual
resets, run ends with a separate update, batch boundaries) are skipped; gated
iterations (pass B < 0.4 of the median) too. One line per launch sequence
(atomic and deterministic runs of one trace are separate lines).
usage: cg_fused_period.py LABEL kernel_trace.csv [LABEL trace ...]"""
import csv
import gzip
import re
import statistics as st
import sys
from collections import defaultdict

ANCHORS = ("k_pass_a_frame", "k_upd_pass_a")


def short(n):
    n = re.sub(r"\(.*", "", n).replace("void ", "").replace("mvba::", "")
    return {"k_point_w_seg": "k_point_w"}.get(re.sub(r"<.*", "", n).strip(), re.sub(r"<.*", "", n).strip())


def periods(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rt") as f:
        ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                    for r in csv.DictReader(f))
    idx = [i for i, e in enumerate(ev) if e[2] in ANCHORS]
    seqs = defaultdict(list)
    for a, b in zip(idx, idx[1:]):
        names = tuple(e[2] for e in ev[a:b])
        if ev[b][2] != ev[a][2] or len(names) != (4 if ev[a][2] == "k_upd_pass_a" else 5) or "k_pass_b" not in names:
            continue  # residual resets, run ends, batch boundaries
        seqs[names].append({"period": (ev[b][0] - ev[a][0]) / 1e3,
                            **{n: (e[1] - e[0]) / 1e3 for n, e in zip(names, ev[a:b])}})
    out = {}
    for names, its in seqs.items():
        med = st.median(i["k_pass_b"] for i in its)
        out[names] = [i for i in its if i["k_pass_b"] >= 0.4 * med]
    return out


def main(args):
    for label, path in zip(args[0::2], args[1::2]):
        for names, its in sorted(periods(path).items(), key=lambda kv: -len(kv[1])):
            busy = sum(st.median(i[k] for i in its) for k in names)
            parts = "  ".join(f"{k.replace('k_', '')} {st.median(i[k] for i in its):6.2f}" for k in names)
            print(f"{label:20s} n={len(its):4d} period {st.median(i['period'] for i in its):7.2f} us"
                  f" (kernels {busy:6.2f}) | {parts}")


if __name__ == "__main__":
    main(sys.argv[1:])
