"""Deterministic mode (mvba_solver_options.deterministic, MVBA_LIN_DETERMINISTIC).

The default solve adds the camera-side entries shared by many frames (a sensor's
extrinsics and intrinsics) with fp64 atomics into replicas, so rounding depends
on arrival order and the eta = 0.1 truncated CG reacts to it (the reference's
own note, rig_calibrator.cc:1913: "The result is more predictable with one
thread"). Deterministic mode stores every contribution in its producer's slab
row and sums each entry in a fixed order.

Checked here: two deterministic linearizations / solves are bit-identical
(normal equations; CG counts, costs and parameters); the deterministic normal
equations equal the oracle's J^T r / J_b^T J_b (1e-9, as tests/test_linearize_gpu.py)
and agree with the atomic path to rounding; a deterministic full solve converges
to the same point as the default one (1e-6, the north_star tolerance)."""
import numpy as np
import pytest
import torch

from multiview_amd import rig
from multiview_amd.evaluator import Evaluator
from oracle.normal_equations import normal_equations_reference

pytestmark = pytest.mark.gpu

TOL = dict(function_tolerance=1e-16, gradient_tolerance=1e-16, parameter_tolerance=1e-12)


def _rig_problem(depth=False, num_points=2000, num_ref=40, seed=5, models=("radtan", "rpc2", "fov")):
    kw = dict(depth_sensors=(2,)) if depth else {}
    R = rig.make_rig(num_sensors=3, num_ref=num_ref, num_points=num_points, obs_per_point=6,
                     models=list(models), seed=seed, **kw)
    F = rig.FloatFlags(camera_poses_to_float=(), intrinsics_to_float=("focal_length", "optical_center",
                                                                       "distortion"),
                       **(dict(depth_tri_weight=10.0, depth_to_image_transforms_to_float=("cam2",), float_scale=True)
                          if depth else {}))
    return rig.build_problem(R, F)


def _linearize(ev, det):
    L = ev.lin_layout()
    t = lambda n: torch.zeros(max(n, 1), dtype=torch.float64, device="cuda")  # noqa: E731
    g, h, pg, ph, c = t(L["cam_grad_size"]), t(L["cam_hess_size"]), t(3 * L["num_points"]), \
        t(6 * L["num_points"]), t(1)
    ev.linearize_device(g, h, pg, ph, c, apply_loss=True, robust_threshold=3.0, deterministic=det)
    ev.sync()
    return [x.cpu().numpy() for x in (g, h, pg, ph, c)]


@pytest.mark.parametrize("depth", [False, True])
def test_deterministic_normal_equations(depth, oracle):
    P = _rig_problem(depth)
    with Evaluator(P) as ev:
        ev.set_params()
        a = _linearize(ev, True)
        b = _linearize(ev, True)
        c = _linearize(ev, False)
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
        for x, y in zip(a, c):
            assert np.allclose(x, y, rtol=1e-12, atol=1e-12 * max(1.0, np.abs(y).max()))
        if not depth:
            _, r_o, J_o = oracle.evaluate(P, oracle.ANALYTIC, apply_loss=True, robust_threshold=3.0)
            g_ref, h_ref, _, _ = normal_equations_reference(P, r_o, J_o, ev.lin_layout())
            assert np.abs(a[0][:g_ref.size] - g_ref).max() <= 1e-9 * max(1.0, np.abs(g_ref).max())
            assert np.abs(a[1][:h_ref.size] - h_ref).max() <= 1e-9 * max(1.0, np.abs(h_ref).max())


@pytest.mark.parametrize("depth", [False, True])
def test_deterministic_solve_is_reproducible(depth):
    # RPC coefficients floated with focal and centre are ill-conditioned (DESIGN.md
    # §4c): the parameter comparison uses well-posed models
    P = _rig_problem(depth, models=("radtan", "fov", "radtan"))
    runs = []
    for _ in range(2):
        with Evaluator(P) as ev:
            ev.set_params()
            s = ev.solve(max_num_iterations=6, use_loss=1, robust_threshold=3.0, deterministic=1, **TOL)
            runs.append((s, ev.get_params()))
    (s0, x0), (s1, x1) = runs
    assert s0["num_linear_iterations"] == s1["num_linear_iterations"]
    assert s0["num_iterations"] == s1["num_iterations"]
    assert s0["final_cost"] == s1["final_cost"]
    assert np.array_equal(x0, x1)
    # the same minimum as the default (atomic) solve
    with Evaluator(P) as ev:
        ev.set_params()
        sd = ev.solve(max_num_iterations=50, use_loss=1, robust_threshold=3.0, **TOL)
        xd = ev.get_params()
        ev.set_params()
        sdet = ev.solve(max_num_iterations=50, use_loss=1, robust_threshold=3.0, deterministic=1, **TOL)
        xdet = ev.get_params()
    assert np.isclose(sdet["final_cost"], sd["final_cost"], rtol=1e-9)
    # |q| of a floated rigid transform (depth_to_image here) is a gauge
    # direction of the cost: compare normalised poses (tests/test_solver_gpu.py)
    from test_solver_gpu import _others, _poses

    assert np.abs(_poses(P, xdet) - _poses(P, xd)).max() <= 1e-6
    o_det, o_d = _others(P, xdet), _others(P, xd)
    assert np.abs(o_det - o_d).max() <= 1e-6 * max(1.0, np.abs(o_d).max())


@pytest.mark.parametrize("depth", [False, True])
def test_graph_replayed_cg_equals_eager(monkeypatch, depth):
    """Single-rank solves replay captured runs of CG iterations (hipGraph,
    mvba_solve.cpp cg_device; MVBA_CG_GRAPH=0 launches every kernel eagerly).
    The captured launches are the eager ones with the same arguments, so in
    deterministic mode the two give bit-identical solves: CG counts, costs,
    parameters. Long enough for the residual reset (every 10th iteration) and
    both parities of the double-buffered vectors, with the captured runs
    replayed across several linear solves of one handle."""
    P = _rig_problem(depth)
    runs = []
    for g in ("0", "1"):
        monkeypatch.setenv("MVBA_CG_GRAPH", g)
        with Evaluator(P) as ev:
            ev.set_params()
            s = ev.solve(max_num_iterations=6, use_loss=1, robust_threshold=3.0, deterministic=1, **TOL)
            runs.append((s, ev.get_params()))
    (sa, xa), (sb, xb) = runs
    assert sa["num_linear_iterations"] > 20, sa["num_linear_iterations"]
    for k in ("termination_type", "num_iterations", "num_successful_steps", "num_linear_iterations", "final_cost"):
        assert sa[k] == sb[k], (k, sa[k], sb[k])
    assert np.array_equal(xa, xb)
