#!/usr/bin/env python3
"""Compare two builds (MVBA_LIB): SHA-256 of the residuals and Jacobian of one
evaluation and of the parameters after a deterministic 3-iteration solve, per
config (c1, the 8-way shard of c2, c2), the arrays kept next to the JSON
(.npz). Run once per build, then --compare A B: identical, or the largest
relative differences (|a - b| / max(|a|, 1)).

usage: MVBA_LIB=... python3 tools/k0_split_check.py --out X.json
       python3 tools/k0_split_check.py --compare A.json B.json
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def h(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--compare", nargs=2)
    a = ap.parse_args()
    if a.compare:
        x, y = (json.load(open(f)) for f in a.compare)
        bad = [k for k in x if x[k] != y.get(k)]
        print("identical" if not bad else f"DIFFERENT: {bad}")
        za, zb = (np.load(f[:-5] + ".npz") for f in a.compare)
        for k in za.files:
            u, v = za[k], zb[k]
            print(f"{k}: max |a - b| / max(|a|, 1) = {(np.abs(u - v) / np.maximum(np.abs(u), 1.0)).max():.3e}")
        sys.exit(0)
    from multiview_amd import rig
    from multiview_amd.evaluator import Evaluator

    out, arrs = {}, {}
    for name, cfg, shard in (("c1", "c1", 1), ("c2_s8", "c2", 8), ("c2", "c2", 1)):
        R = rig.make_rig(**dict(rig.CONFIGS[cfg]))
        if shard > 1:
            R = rig.shard_points(R, 0, shard)
        P = rig.build_problem(R, rig.FloatFlags(**rig.CONFIG_FLAGS.get(cfg, {})))
        with Evaluator(P) as ev:
            ev.set_params()
            cost, r, J = ev.evaluate(True)
            ev.solve(max_num_iterations=3, deterministic=1)
            x3 = ev.get_params()
        for k, v in (("res", r), ("jac", J), ("x3", x3)):
            out[f"{name}_{k}"] = h(v)
            arrs[f"{name}_{k}"] = v[:: max(1, v.size // 250000)]  # every row of c1, a sample of c2's
        print(name, {k: v for k, v in out.items() if k.startswith(name + "_")}, flush=True)
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)
        np.savez(a.out[:-5] + ".npz", **arrs)


if __name__ == "__main__":
    main()
