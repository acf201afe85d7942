"""Which CG direction form drifts? On the problem of
tests/test_solver_forms_gpu.py::test_cg_direction_forms_agree, each form's
eta = 1e-14 step is compared with the CPU exact step of the same damped,
Jacobi-scaled system (oracle/lm_reference.first_step_system), and its relative
normal-equation residual ||A y - b|| / ||b|| is reported beside kappa(A).
Optional: MVBA_CG_WP_RESET values are swept too (argv)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from multiview_amd import rig  # noqa: E402
from multiview_amd.evaluator import Evaluator  # noqa: E402
from oracle import lm_reference  # noqa: E402

R = rig.make_rig(num_sensors=3, num_ref=40, num_points=3000, obs_per_point=6, seed=13)
P = rig.build_problem(R, rig.FloatFlags(camera_poses_to_float=()))
tol = dict(function_tolerance=1e-16, gradient_tolerance=1e-16, parameter_tolerance=1e-12)
sysm = lm_reference.first_step_system(P, use_loss=True, robust_threshold=3.0)
A, b, s, idx, ys = sysm["A"], sysm["b"], sysm["s"], sysm["idx"], sysm["y_exact"]
print(f"n={idx.size} lam_max={sysm['lam_max']:.3e} lam_min={sysm['lam_min']:.3e} kappa={sysm['kappa']:.3e} "
      f"exact residual {np.linalg.norm(A @ ys - b) / np.linalg.norm(b):.2e}", flush=True)
for form in sys.argv[1:] or ["0", "1"]:
    os.environ["MVBA_CG_DIR_KERNEL"] = form
    for eta in (1e-14,):
        with Evaluator(P) as ev:
            ev.set_params()
            st = ev.solve(max_num_iterations=1, eta=eta, max_linear_solver_iterations=4000, use_loss=1,
                          robust_threshold=3.0, **tol)
            x = ev.get_params()
        y = (x[idx] - sysm["x0"]) / s
        res = np.linalg.norm(A @ y - b) / np.linalg.norm(b)
        err = np.linalg.norm(y - ys) / np.linalg.norm(ys)
        scale = np.maximum(np.abs(x[idx]), 1.0)
        xe = sysm["x0"] + s * ys
        print(f"form {form} eta {eta:.0e}: cg {st['num_linear_iterations']} residual {res:.3e} err {err:.3e} "
              f"(bound kappa*res {sysm['kappa'] * res:.3e}) max param rel {(np.abs(x[idx] - xe) / scale).max():.3e}",
              flush=True)
