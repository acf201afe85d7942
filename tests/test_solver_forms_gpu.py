"""Size-selected forms of the solver passes, forced both ways on one problem.

* Where pass A leaves c_o = J_pt^T z_o (MVBA_CO_ORDER): at the observation's
  point-order position (scattered stores, the default below 128 MB of table)
  or in slot order with k_point_w gathering through po_slot (c3 and up). The
  point solve sums in the same point order either way, so a deterministic
  solve is bit-identical in both forms.
* The back-substitution's |J delta|^2 (MVBA_BACKSUB): the point-order pass
  (depth blocks, XYZ priors, several models) or frame-order pass A + k_point_w
  + k_pass_sq (reprojection-only problems, the default). Same quantities
  summed in another order: the solves agree to rounding.

Both variables are read at every call, so one process runs both forms."""
import numpy as np
import pytest

from multiview_amd import rig
from multiview_amd.evaluator import Evaluator


def _problem():
    R = rig.make_rig(num_sensors=3, num_ref=10, num_points=400, obs_per_point=4, seed=11)
    return rig.build_problem(R)


def _solve(P, **kw):
    with Evaluator(P) as ev:
        ev.set_params()
        s = ev.solve(max_num_iterations=4, use_loss=1, robust_threshold=3.0, deterministic=1, **kw)
        return s, ev.get_params()


@pytest.mark.gpu
def test_co_order_forms_bit_identical(monkeypatch):
    P = _problem()
    runs = []
    for order in ("point", "slot"):
        monkeypatch.setenv("MVBA_CO_ORDER", order)
        runs.append(_solve(P))
    (sa, xa), (sb, xb) = runs
    for k in ("termination_type", "num_iterations", "num_successful_steps", "num_linear_iterations", "final_cost"):
        assert sa[k] == sb[k], (k, sa[k], sb[k])
    assert np.array_equal(xa, xb)


@pytest.mark.gpu
def test_back_substitution_forms_agree(monkeypatch):
    P = _problem()
    runs = []
    for form in ("point", "frame"):
        monkeypatch.setenv("MVBA_BACKSUB", form)
        runs.append(_solve(P))
    (sa, xa), (sb, xb) = runs
    for k in ("num_iterations", "num_successful_steps"):
        assert sa[k] == sb[k], (k, sa[k], sb[k])
    assert sa["final_cost"] < sa["initial_cost"]
    assert np.isclose(sa["final_cost"], sb["final_cost"], rtol=1e-9), (sa["final_cost"], sb["final_cost"])
    scale = np.maximum(np.abs(xa), 1.0)
    assert (np.abs(xa - xb) / scale).max() < 1e-7


@pytest.mark.gpu
def test_cg_direction_forms_agree(monkeypatch):
    """The CG direction records (MVBA_CG_DIR_KERNEL, read per call): the
    default forms W p as W z + beta W p_old (the update kernel's FrameDirZ
    blocks + pass A's DirPair writer) and the direction-kernel form computes
    W (z + beta p_old) in k_frame_dir: the same quantities rounded in another
    order. The problem is sized so linear solves run past 10 CG iterations,
    i.e. through Ceres' residual reset (i % residual_reset_period == 0).
    * one LM iteration with CG run to convergence: both forms give the exact
      step (1e-8 relative);
    * default truncated CG (eta = 0.1), solved to Ceres' tolerances: both reach
      the same minimum (cost rtol 1e-9, parameters 1e-6). Mid-solve costs are
      not comparable: a rounding change moves the truncated CG's stopping
      point and with it the LM path."""
    R = rig.make_rig(num_sensors=3, num_ref=40, num_points=3000, obs_per_point=6, seed=13)
    # reference poses fixed: a unique minimum (with every pose floating the
    # gauge directions leave the damped system too ill-conditioned for two
    # roundings of CG to agree to 1e-8)
    Pc = rig.build_problem(R, rig.FloatFlags(camera_poses_to_float=()))
    P = Pc
    tol = dict(function_tolerance=1e-16, gradient_tolerance=1e-16, parameter_tolerance=1e-12)
    exact, conv = [], []
    for form in ("0", "1"):
        monkeypatch.setenv("MVBA_CG_DIR_KERNEL", form)
        with Evaluator(P) as ev:
            ev.set_params()
            s = ev.solve(max_num_iterations=1, eta=1e-14, max_linear_solver_iterations=4000, use_loss=1,
                         robust_threshold=3.0, **tol)
            exact.append((s, ev.get_params()))
        with Evaluator(Pc) as ev:
            ev.set_params()
            s = ev.solve(max_num_iterations=200, use_loss=1, robust_threshold=3.0, **tol)
            conv.append((s, ev.get_params()))
    (sa, xa), (sb, xb) = exact
    assert sa["num_linear_iterations"] > 10 and sb["num_linear_iterations"] > 10
    # CG to eta = 1e-14 on this 3,000-landmark problem: the two roundings
    # agree to the system's conditioning (measured 3e-8 with frames in first-use
    # order, 1.2e-7 in capture order: profiles/r04/r04m/pytest_gpu_r04m.log)
    scale = np.maximum(np.abs(xa), 1.0)
    assert (np.abs(xa - xb) / scale).max() < 5e-7
    (sa, xa), (sb, xb) = conv
    assert sa["termination_type"] == 0 and sb["termination_type"] == 0, (sa["message"], sb["message"])
    # the same minimum: the cost to rounding (some intrinsics / rig directions of
    # this rig are nearly flat, so converged parameters differ there by up to
    # 2e-3 at costs equal to 1e-9, as two CPU runs with different radii do:
    # tests/test_solver_gpu.py::test_ill_conditioned_rpc_reaches_same_cost)
    assert np.isclose(sa["final_cost"], sb["final_cost"], rtol=1e-9), (sa["final_cost"], sb["final_cost"])
