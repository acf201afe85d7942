"""One LM solve at a bench configuration (default c2, 5 iterations, all blocks
floating, Cauchy 3.0): a short program for kernel traces and A/B runs.

    python tools/solve_probe.py [--config c2] [--iters 5] [--deterministic]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from multiview_amd import rig  # noqa: E402
from multiview_amd.evaluator import Evaluator  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--deterministic", action="store_true")
a = ap.parse_args()
R = rig.make_rig(**dict(rig.CONFIGS[a.config]))
P = rig.build_problem(R, rig.FloatFlags(**rig.CONFIG_FLAGS.get(a.config, {})))
kw = dict(max_num_iterations=a.iters, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0,
          use_loss=1, robust_threshold=3.0, deterministic=int(a.deterministic))
with Evaluator(P) as ev:
    ev.set_params()
    ev.solve(**dict(kw, max_num_iterations=1))
    ev.set_params()
    t = time.perf_counter()
    s = ev.solve(**kw)
    dt = time.perf_counter() - t
    print(f"{a.config}: {s['num_iterations']} LM iterations, {s['num_linear_iterations']} CG, {dt * 1e3:.1f} ms, "
          f"{1e3 * s['linear_solver_time_s'] / max(s['num_linear_iterations'], 1) * 1e3:.1f} us/CG", flush=True)
