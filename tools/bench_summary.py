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
        out = [path.split("/")[-1], f"{r.get('kernel', 'K1')} {r['kernel_ms'] * 1e3:.1f} us",
               f"{r['achieved']:.0f} GB/s", f"frac {r['frac']:.3f}", f"evals/s {d['value']:.3g}",
               f"step {d['ms_per_step'] * 1e3:.1f} us"]
        if "split_form" in r:
            out.append(f"split K1 {r['split_form']['kernel_ms'] * 1e3:.1f} us (frac {r['split_form']['frac']:.3f})")
        if "cpu_baseline" in d:
            out.append(f"cpu {d['cpu_baseline']['value']:.3g} evals/s ({d['cpu_baseline']['cores']} thr)")
        if "eval_f32" in d:
            e = d["eval_f32"]
            out.append(f"f32 {e['kernel_ms'] * 1e3:.1f} us {e['achieved_GBps']:.0f} GB/s")
        if "depth" in d:
            e = d["depth"]
            out.append("depth " + " ".join(f"{k}={v:.4g}" for k, v in e.items() if isinstance(v, float))[:160])
        if d.get("linearize") and "kernel_ms" in d["linearize"]:
            out.append(f"lin {d['linearize']['kernel_ms'] * 1e3:.1f} us")
        if "ba" in d and "iters_per_s" in d["ba"]:
            cg = d['ba'].get('ms_per_cg_iteration')
            out.append(f"LM {d['ba']['iters_per_s']:.1f} it/s ({d['ba']['cg_iterations']} CG"
                       + (f", {1e3 * cg:.0f} us/CG)" if cg else ")"))
        print(" | ".join(out))
