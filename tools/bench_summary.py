#!/usr/bin/env python3
"""One line per bench.py log: K1 time, algorithmic GB/s, roofline fraction, and
the optional phase numbers (fp32 outputs, depth, linearize, LM)."""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        r = d["roofline"]
        out = [path.split("/")[-1], f"K1 {r['kernel_ms'] * 1e3:.1f} us", f"{r['achieved']:.0f} GB/s",
               f"frac {r['frac']:.3f}", f"evals/s {d['value']:.3g}"]
        if "eval_f32" in d:
            e = d["eval_f32"]
            out.append(f"f32 {e['kernel_ms'] * 1e3:.1f} us {e['achieved_GBps']:.0f} GB/s")
        if "depth" in d:
            e = d["depth"]
            out.append("depth " + " ".join(f"{k}={v:.4g}" for k, v in e.items() if isinstance(v, float))[:160])
        if "linearize" in d:
            out.append(f"lin {d['linearize']['kernel_ms'] * 1e3:.1f} us")
        if "ba" in d:
            cg = d['ba'].get('ms_per_cg_iteration')
            out.append(f"LM {d['ba']['iters_per_s']:.1f} it/s ({d['ba']['cg_iterations']} CG"
                       + (f", {1e3 * cg:.0f} us/CG)" if cg else ")"))
        print(" | ".join(out))
