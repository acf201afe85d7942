"""XYZError priors (rig_calibrator.cc:709-751; --tri_weight, :1889-1898).

CPU: the constructor's block-size check in mvba_create. GPU: residuals /
Jacobian / cost against the oracle restatement, their point-side normal
equations, and the LM with priors: one exact step against the dense CPU LM and
converged parameters (the prior keeps points near their start values, so even
with every pose floating the minimum is unique up to the quaternion-norm gauge)."""
import numpy as np
import pytest

from multiview_amd import _lib, rig
from multiview_amd.evaluator import Evaluator
from oracle.normal_equations import normal_equations_reference

TOL = dict(function_tolerance=1e-16, gradient_tolerance=1e-16, parameter_tolerance=1e-12)


def _problem(seed=5, **flags):
    R = rig.make_rig(num_sensors=3, num_ref=12, num_points=200, obs_per_point=5, models=["radtan", "fov", "none"],
                     seed=seed)
    f = dict(tri_weight=0.5, tri_robust_threshold=0.1)
    f.update(flags)
    return R, rig.build_problem(R, rig.FloatFlags(**f))


def test_xyz_block_size_check_before_device():
    _, P = _problem()
    P.xyz_block = P.xyz_block.copy()
    P.xyz_block[0] = 0  # a 7-parameter pose block
    with pytest.raises(_lib.MvbaError) as e:
        Evaluator(P)
    assert e.value.status == _lib.MVBA_E_XYZ_BLOCK_SIZES


@pytest.mark.gpu
@pytest.mark.parametrize("apply_loss", [False, True])
def test_xyz_eval_parity(oracle, apply_loss):
    _, P = _problem()
    P.params = P.params.copy()
    P.params[P.block_offset[P.xyz_block[0]]] += 0.3  # move one point off its prior
    with Evaluator(P) as ev:
        ev.set_params()
        c, r, J = ev.evaluate_xyz(jacobian=True, apply_loss=apply_loss)
    c_o, r_o, J_o = oracle.evaluate_xyz(P, apply_loss=apply_loss)
    assert np.isclose(c, c_o, rtol=1e-12, atol=1e-300)
    assert np.abs(r - r_o).max() <= 1e-12 * max(np.abs(r_o).max(), 1.0)
    assert np.abs(J - J_o).max() <= 1e-12 * np.abs(J_o).max()


@pytest.mark.gpu
def test_xyz_linearize_parity(oracle):
    import torch

    _, P = _problem(seed=6)
    P.params = P.params.copy()
    P.params[P.block_offset[P.xyz_block]] += np.linspace(-0.2, 0.2, P.num_xyz_residuals)
    with Evaluator(P) as ev:
        ev.set_params()
        L = ev.lin_layout()
        t = lambda n: torch.zeros(n, dtype=torch.float64, device="cuda")  # noqa: E731
        cg, ch, pg, ph, cost = t(L["cam_grad_size"]), t(L["cam_hess_size"]), t(3 * L["num_points"]), \
            t(6 * L["num_points"]), t(1)
        ev.linearize_device(cg, ch, pg, ph, cost, apply_loss=True, robust_threshold=3.0)
        ev.sync()
    c_o, r_o, J_o = oracle.evaluate(P, oracle.ANALYTIC, apply_loss=True, robust_threshold=3.0)
    g, h, pgr, phr = normal_equations_reference(P, r_o, J_o, L)
    cx, rx, Jx = oracle.evaluate_xyz(P, apply_loss=True)
    pos = {int(b): k for k, b in enumerate(L["point_block_ids"])}
    pgr = pgr.reshape(-1, 3)
    phr = phr.reshape(-1, 6)
    for j in range(P.num_xyz_residuals):
        k = pos[int(P.xyz_block[j])]
        Jj = Jx[j].reshape(3, 3)
        pgr[k] += Jj.T @ rx[j]
        H = Jj.T @ Jj
        phr[k] += H[[0, 0, 0, 1, 1, 2], [0, 1, 2, 1, 2, 2]]
    got_g = pg.cpu().numpy().reshape(-1, 3)
    got_h = ph.cpu().numpy().reshape(-1, 6)
    assert (np.abs(got_g - pgr) <= 1e-9 * np.maximum(np.abs(pgr).max(axis=1, keepdims=True), 1e-300)).all()
    assert (np.abs(got_h - phr) <= 1e-9 * np.maximum(np.abs(phr).max(axis=1, keepdims=True), 1e-300)).all()
    assert np.isclose(cost.item(), c_o + cx, rtol=1e-11)


@pytest.mark.gpu
def test_xyz_solver_one_exact_step_and_convergence():
    from oracle import lm_reference

    _, P = _problem(seed=7, camera_poses_to_float=())
    x_ref, s_ref = lm_reference.solve(P, max_num_iterations=1, use_loss=True, **TOL)
    with Evaluator(P) as ev:
        ev.set_params()
        s = ev.solve(max_num_iterations=1, eta=1e-14, max_linear_solver_iterations=2000, use_loss=1,
                     robust_threshold=3.0, **TOL)
        x = ev.get_params()
    assert np.isclose(s["initial_cost"], s_ref["initial_cost"], rtol=1e-11)
    assert np.abs(x - x_ref).max() <= 1e-8 * max(1.0, np.abs(x_ref).max())
    x_ref, s_ref = lm_reference.solve(P, max_num_iterations=100, use_loss=True, **TOL)
    with Evaluator(P) as ev:
        ev.set_params()
        s = ev.solve(max_num_iterations=200, use_loss=1, robust_threshold=3.0, **TOL)
    assert s["termination_type"] == 0, s["message"]
    assert np.isclose(s["final_cost"], s_ref["final_cost"], rtol=1e-9)
