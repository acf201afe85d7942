#!/usr/bin/env python3
"""Repeat the single-observation-points solve of tests/test_edge_cases.py a few
times in one process: termination reason and final cost against the CPU LM
(the fp64 atomics make the last rounding-level steps differ run to run)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from multiview_amd import rig
    from multiview_amd.evaluator import Evaluator
    from oracle import lm_reference

    R = rig.make_rig(num_sensors=3, num_ref=8, num_points=150, obs_per_point=2.0, models=["radtan", "fov", "none"],
                     seed=21)
    P = rig.build_problem(R, rig.FloatFlags(camera_poses_to_float=()))
    keep = np.ones(P.num_residuals, bool)
    first = np.r_[True, R.obs_pid[1:] != R.obs_pid[:-1]]
    keep[~first] = np.arange((~first).sum()) % 2 == 0
    for name in ("residual_blocks", "residual_camera", "residual_meas", "residual_stamps"):
        setattr(P, name, getattr(P, name)[keep])
    P.residual_names = None
    TOL = dict(function_tolerance=1e-16, gradient_tolerance=1e-16, parameter_tolerance=1e-12)
    _, s_ref = lm_reference.solve(P, max_num_iterations=100, use_loss=True, **TOL)
    print("cpu LM", s_ref["final_cost"], flush=True)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    for det in (0, 1):
      for k in range(reps):
        with Evaluator(P) as ev:
            ev.set_params()
            s = ev.solve(max_num_iterations=200, use_loss=1, robust_threshold=3.0, deterministic=det, **TOL)
        print("det" if det else "atomic", k, s["termination_type"], s["num_iterations"],
              s["num_successful_steps"], s["num_linear_iterations"], "%.17g" % s["final_cost"],
              "rel %.2e" % abs(s["final_cost"] / s_ref["final_cost"] - 1), s["message"][:70], flush=True)


if __name__ == "__main__":
    main()
