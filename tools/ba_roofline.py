#!/usr/bin/env python3
"""Committed summary of one CG iteration (the BA half of the metric) from a
rocprofv3 kernel trace and the separate --pmc passes of the same bench command.

usage: ba_roofline.py OUT.json CONFIG kernel_trace.csv fetch.csv write.csv sq.csv [l2.csv]

A CG iteration of a reprojection-only problem is the launch sequence
    k_pass_a_frame -> k_point_w -> k_pass_b -> k_vec_rep_reduce -> k_cg_update
(the fused-direction CG; a k_frame_dir in front marks a residual-reset or
right-hand-side product, which is skipped), or, with the fused CG step (the
default below 400k observations: thin shards),
    k_upd_pass_a -> k_point_w -> k_pass_b -> k_vec_rep_reduce (-> k_upd_pass_a)
whichever the trace holds more of. Iterations whose pass B ran (gated
launches past the CG stop take ~2-5 us) give
  kernel_us      median over iterations of end(k_cg_update) - start(k_pass_a_frame),
                 or for the fused step start(next k_upd_pass_a) - start(k_upd_pass_a)
                 (kernel boundaries included), and the per-kernel medians;
from the PMC passes, per kernel, the median over its launches in the upper
half (the non-gated ones):
  FETCH_SIZE x 2 (gfx950 tallies 128-B requests at 64 B, MI355X_MICROARCH.md
  HBM section) + WRITE_SIZE -> traffic bytes, SQ_INSTS_VALU -> issue floor
  (4 cycles per fp64 wave instruction on one of 1,024 SIMDs at 2.4 GHz);
  with l2.csv (TCC_HIT_sum, TCC_MISS_sum) the L2 hit rate per kernel.
bench.py reads OUT.json for ba.roofline's kernel time, traffic and VALU floor.
"""
import csv
import json
import re
import statistics as st
import sys
from collections import defaultdict

SEQ = ["k_pass_a_frame", "k_point_w", "k_pass_b", "k_vec_rep_reduce", "k_cg_update"]
SEQ_FUSED = ["k_upd_pass_a", "k_point_w", "k_pass_b", "k_vec_rep_reduce"]


def short(name):
    name = re.sub(r"\(.*", "", name).replace("void ", "").replace("mvba::", "")
    name = re.sub(r"<.*", "", name).strip()
    return {"k_point_w_seg": "k_point_w"}.get(name, name)  # the point solve's tile form


def trace_iterations(path, seq=None):
    """Non-gated CG iterations of the trace: (iterations, launch sequence).
    seq None: the form the trace holds more iterations of."""
    if seq is None:
        a, b = trace_iterations(path, SEQ), trace_iterations(path, SEQ_FUSED)
        return b if len(b[0]) > len(a[0]) else a
    ev = []
    with open(path) as f:
        for r in csv.DictReader(f):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    ev.sort()
    fused = seq[0] == "k_upd_pass_a"
    groups = []
    for i in range(1, len(ev) - len(seq)):
        if [e[2] for e in ev[i:i + len(seq)]] != seq or ev[i - 1][2] == "k_frame_dir":
            continue
        if fused and ev[i + len(seq)][2] != "k_upd_pass_a":
            continue  # the fused step's period ends at the next fused launch
        groups.append((ev[i:i + len(seq)], ev[i + len(seq)]))
    if not groups:
        return [], seq
    # gated iterations (past the CG stop) return at once: their pass B is a
    # small fraction of a working one's (any chunking, any problem size)
    pbs = sorted(g[0][2][1] - g[0][2][0] for g in groups)
    pb_ref = pbs[len(pbs) // 2]
    its = []
    for grp, nxt in groups:
        if (grp[2][1] - grp[2][0]) < 0.4 * pb_ref:
            continue
        span = (nxt[0] - grp[0][0]) if fused else (grp[-1][1] - grp[0][0])
        its.append({"span_us": span / 1e3, **{k: (e[1] - e[0]) / 1e3 for k, e in zip(seq, grp)}})
    return its, seq


def pmc(paths, seq=SEQ):
    d = defaultdict(lambda: defaultdict(list))
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                d[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k in seq:
        row = {}
        for c, v in d[k].items():
            v = sorted(v)[len(v) // 2:]
            row[c] = st.median(v)
        out[k] = row
    return out


def main():
    out, cfg, trace, fetch, write, sq = sys.argv[1:7]
    extra = [a for a in sys.argv[7:8] if a]
    its, seq = trace_iterations(trace)
    if not its:
        raise SystemExit("no non-gated CG iterations in the trace")
    counters = pmc([fetch, write, sq] + extra, seq)
    per_k = {}
    traffic = valu = 0.0
    for k in seq:
        c = counters[k]
        fb = 2e3 * c.get("FETCH_SIZE", 0.0)  # KB -> bytes, x2 (gfx950 FETCH_SIZE)
        wb = 1e3 * c.get("WRITE_SIZE", 0.0)
        per_k[k] = {"us": st.median(i[k] for i in its), "fetch_bytes": fb, "write_bytes": wb,
                    "valu_insts": c.get("SQ_INSTS_VALU"), "waves": c.get("SQ_WAVES")}
        for name, key in (("wait_frac", "SQ_WAIT_ANY"), ("active_frac", "SQ_ACTIVE_INST_ANY")):
            if c.get("SQ_WAVE_CYCLES"):
                per_k[k][name] = c.get(key, 0.0) / c["SQ_WAVE_CYCLES"]
        if c.get("TCC_HIT_sum") is not None and c.get("TCC_MISS_sum") is not None:
            tot = c["TCC_HIT_sum"] + c["TCC_MISS_sum"]
            per_k[k]["l2_hit"] = c["TCC_HIT_sum"] / tot if tot else None
        traffic += fb + wb
        valu += c.get("SQ_INSTS_VALU", 0.0)
    res = {
        "config": cfg,
        "generator": "tools/ba_roofline.py",
        "iterations_used": len(its),
        "cg_form": "fused step" if seq[0] == "k_upd_pass_a" else "separate update",
        "kernel_us_per_cg_iteration": st.median(i["span_us"] for i in its),
        "traffic_bytes_per_cg_iteration": traffic,
        "valu_insts_per_cg_iteration": valu,
        "valu_floor_us": valu * 4 / (1024 * 2.4e9) * 1e6,
        "kernels": per_k,
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))
    for k, v in per_k.items():
        print(f"{k:18s} {v['us']:7.2f} us  fetch {v['fetch_bytes'] / 1e6:7.2f} MB  write {v['write_bytes'] / 1e6:7.2f} MB"
              f"  valu {v['valu_insts'] or 0:10.0f}  wait {v.get('wait_frac', 0):.2f}  l2hit {v.get('l2_hit') or 0:.2f}")


if __name__ == "__main__":
    main()
