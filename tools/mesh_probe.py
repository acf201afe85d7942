"""Repeat the depth-mesh exact-step case of tests/test_mesh.py and print, per
run, the CG count and the largest deviation from the dense LM step (is the
deviation run-to-run, and does deterministic mode remove it?)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
from multiview_amd import rig
from multiview_amd.evaluator import Evaluator
from oracle import lm_reference
from test_mesh import _sphere_rig, _mesh_flags, _oracle_mesh_xyz
from test_solver_gpu import TOL, _free_mask
from test_solver_forms_gpu import _check_against_exact_step

R = _sphere_rig(seed=21, num_ref=16, num_points=300)
P = rig.build_problem(R, _mesh_flags(camera_poses_to_float=()), mesh_xyz=_oracle_mesh_xyz(R))
m = _free_mask(P)
for use_loss in (False, True):
    x_ref, s_ref = lm_reference.solve(P, max_num_iterations=1, use_loss=use_loss, **TOL)
    sysm = lm_reference.first_step_system(P, use_loss=use_loss)
    for det in (0, 1):
        for rep in range(12 if det == 0 else 2):
            with Evaluator(P) as ev:
                ev.set_params()
                s = ev.solve(max_num_iterations=1, eta=1e-14, max_linear_solver_iterations=2000,
                             use_loss=int(use_loss), robust_threshold=3.0, deterministic=det, **TOL)
                x = ev.get_params()
            d = np.abs(x[m] - x_ref[m])
            print(f"loss={int(use_loss)} det={det} rep={rep} cg={s['num_linear_iterations']} "
                  f"dev={d.max():.3e} at {np.argmax(d)} |x|={np.abs(x_ref[m]).max():.3g} cost={s['final_cost']:.12g} ref={s_ref['final_cost']:.12g}", flush=True)
            try:
                _check_against_exact_step(sysm, x, f"  loss={int(use_loss)} det={det}")
            except AssertionError as e:
                print("  EXACT-STEP CHECK FAILED", e, flush=True)
