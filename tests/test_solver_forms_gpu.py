"""Size-selected forms of the solver passes, forced both ways on one problem.

* Where pass A leaves c_o = J_pt^T z_o (MVBA_CO_ORDER): at the observation's
  point-order position (scattered stores, the default below 128 MB of table)
  or in slot order with k_point_w gathering through po_slot (c3 and up). The
  point solve sums in the same point order either way, so a deterministic
  solve is bit-identical in both forms.
* The back-substitution's |J delta|^2 (MVBA_BACKSUB): the point-order pass
  (depth blocks, XYZ priors, several models) or frame-order pass A + k_point_w
  + k_pass_sq (reprojection-only problems, the default). Same quantities
  summed in another order: one LM step agrees to rounding.
* The point solve w_p = (V + D)^-1 (t + sum c_o) (MVBA_POINT_W): wave tiles of
  whole tracks (k_point_w_seg) or 8 lanes per point (k_point_w).

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


def _one_step(P, **kw):
    """One LM step with the CG run to eta = 1e-14, deterministic sums: every
    form under test then starts from the same camera step, so the forms of the
    point solve / back-substitution are compared on one step, where they must
    agree to rounding. (Several LM steps compare trajectories instead: a
    rounding-level difference moves the truncated CG's stopping point, and
    the costs after 4 steps of a non-converged solve then differ by 1e-4
    relative without any error, as profiles/r04/r04u's 219.8999 vs 219.9178.)"""
    with Evaluator(P) as ev:
        ev.set_params()
        s = ev.solve(max_num_iterations=1, eta=1e-14, max_linear_solver_iterations=2000, use_loss=1,
                     robust_threshold=3.0, deterministic=1, function_tolerance=1e-16, gradient_tolerance=1e-16,
                     parameter_tolerance=1e-16, **kw)
        return s, ev.get_params()


def _exact_step_system(P):
    from oracle import lm_reference

    return lm_reference.first_step_system(P, use_loss=True, robust_threshold=3.0)


def _check_against_exact_step(sysm, x, label, param_tol=1e-6):
    """A GPU step against the CPU's exact step of the same damped, Jacobi-
    scaled normal equations A y = b (lm_reference.first_step_system): the
    relative residual <= 1e-8 (CG at eta = 1e-14 solved the system), the
    error within kappa(A) x residual (true for any SPD system: the two sides
    solved the same system) and every free parameter within param_tol = 1e-6
    relative of the exact step (north_star's parity bound).

    param_tol None: the per-parameter error is reported against 1e-6 and held
    to the bound the residual implies instead, |dx|_inf <= |s|_inf x kappa x
    res x |y|_2 (x = x0 + s y): for a CG whose stopping point moves with the
    order of its fp64 sums on an ill-conditioned system (the atomic path). The
    return value is that error."""
    A, b, sc, idx, ys, kappa = sysm["A"], sysm["b"], sysm["s"], sysm["idx"], sysm["y_exact"], sysm["kappa"]
    x_exact = sysm["x0"] + sc * ys
    y = (x[idx] - sysm["x0"]) / sc
    res = np.linalg.norm(A @ y - b) / np.linalg.norm(b)
    err = np.linalg.norm(y - ys) / np.linalg.norm(ys)
    perr = (np.abs(x[idx] - x_exact) / np.maximum(np.abs(x_exact), 1.0)).max()
    implied = np.abs(sc).max() * kappa * res * np.linalg.norm(ys) * (1 + 1e-6) + 1e-14
    print(f"{label}: residual {res:.2e}, error {err:.2e} (kappa {kappa:.2e}), max parameter error {perr:.2e} "
          f"({'within' if perr <= 1e-6 else 'ABOVE'} 1e-6; residual-implied bound {implied:.2e})")
    assert res <= 1e-8, (label, res)
    assert err <= kappa * res * (1 + 1e-6) + 1e-14, (label, err, kappa * res)
    if param_tol is None:
        assert np.abs(x[idx] - x_exact).max() <= implied, (label, np.abs(x[idx] - x_exact).max(), implied)
    else:
        assert perr <= param_tol, (label, perr)
    return perr


def _agree(a, b, tol, same_cg=True):
    (sa, xa), (sb, xb) = a, b
    for k in ("num_iterations", "num_successful_steps") + (("num_linear_iterations",) if same_cg else ()):
        assert sa[k] == sb[k], (k, sa[k], sb[k])
    assert sa["final_cost"] < sa["initial_cost"]
    assert np.isclose(sa["final_cost"], sb["final_cost"], rtol=tol, atol=0), (sa["final_cost"], sb["final_cost"])
    scale = np.maximum(np.abs(xa), 1.0)
    assert (np.abs(xa - xb) / scale).max() <= tol, (np.abs(xa - xb) / scale).max()


@pytest.mark.gpu
def test_back_substitution_forms_agree(monkeypatch):
    """The point-order back-substitution pass and the frame-order one (pass A +
    k_point_w + k_pass_sq) on the same step: same point updates and model cost
    change to rounding (parameters and cost 1e-12 relative)."""
    P = _problem()
    runs = []
    for form in ("point", "frame"):
        monkeypatch.setenv("MVBA_BACKSUB", form)
        runs.append(_one_step(P))
    _agree(runs[0], runs[1], 1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("long_tracks", [False, True])
def test_point_solve_forms_agree(monkeypatch, long_tracks):
    """k_point_w's two forms (MVBA_POINT_W, read per call): wave tiles of whole
    tracks with a segmented lane scan (k_point_w_seg) and 8 lanes per point
    with lane-strided gathers (k_point_w). Same sums in another order: one LM
    step (CG products and back-substitution both use the form) agrees to
    rounding. long_tracks: most tracks exceed a wave (65..90 residuals), so
    their tiles take the lane-strided loop and wave sum; the rest share tiles."""
    if long_tracks:
        R = rig.make_rig(num_sensors=3, num_ref=60, num_points=300, obs_per_point=90, window=30, seed=3)
        assert (np.bincount(R.obs_pid) > 64).sum() > 100
    else:
        R = rig.make_rig(num_sensors=3, num_ref=10, num_points=400, obs_per_point=4, seed=11)
    # reference poses fixed: a unique minimum, so each form's step can be held
    # against the CPU's exact step (the CG products use the form too, so the
    # two forms' eta = 1e-14 stopping points differ; with every pose floating
    # the gauge directions put them 1.1e-7 apart, profiles/r05/r05h/)
    P = rig.build_problem(R, rig.FloatFlags(camera_poses_to_float=()))
    sysm = _exact_step_system(P)
    for form in ("lanes", "tiles"):
        monkeypatch.setenv("MVBA_POINT_W", form)
        s, x = _one_step(P)
        assert s["final_cost"] < s["initial_cost"]
        _check_against_exact_step(sysm, x, form)


@pytest.mark.gpu
def test_cg_direction_forms_agree(monkeypatch):
    """The CG direction records (MVBA_CG_DIR_KERNEL, MVBA_CG_DZ, read per
    call): the default forms W p as W z + beta W p_old with W z from the CG
    update kernel's frame blocks (FrameDirZ) and pass A keeping W p for the
    next product (DirPair writer); the fused CG step (MVBA_CG_FUSE,
    k_upd_pass_a) runs the update inside the next pass A, which forms W z
    itself and both products (c_z, c_p) for k_point_w to combine with beta,
    whose frame blocks store W p; MVBA_CG_DZ=passa has pass A form the pose
    sums W z of its frame from z (DirPair::frec) instead; the direction-kernel form
    computes W (z + beta p_old) in k_frame_dir. The problem is sized so linear
    solves run past 10 CG iterations, i.e. through Ceres' residual reset.

    Each form is checked against the CPU's exact step, not against the other
    form: oracle/lm_reference.first_step_system builds the first LM
    iteration's damped, Jacobi-scaled normal equations A y = b (the system
    both the CPU LM and the GPU's Schur-CG solve; SPD, kappa(A) from its
    extreme eigenvalues) and the GPU step delta = S y is mapped into it.
    * CG at eta = 1e-14 must solve the normal equations: relative residual
      ||A y - b|| / ||b|| <= 1e-8 for both forms. The q-criterion stops on the
      quadratic model's decrease, not on the residual: measured 2e-10 (kernel
      form) and 7e-10 (recurrence form), 87-89 CG iterations
      (profiles/r05/r05b/cg_probe_r05b.log, tools/cg_form_probe.py);
    * the step's error against the exact step obeys ||y - y*|| / ||y*|| <=
      kappa(A) * residual (true for any SPD system: the GPU and the CPU solved
      the same system), and every free parameter is within 1e-6 relative of
      the exact step (north_star's parity bound). Measured 3e-8 / 4e-8 of
      ||y*|| (kappa 8.7e4), max parameter error 1.3e-8 / 1.6e-8: neither form
      drifts. Round 4 compared the forms with each other at 1e-8 relative and
      saw 1.2e-7: that is the sum of two such errors, not a drift;
    * default truncated CG (eta = 0.1) solved to Ceres' tolerances: both reach
      the same minimum cost (rtol 1e-9). Converged parameters are not
      compared: some intrinsics / rig directions of this rig are nearly flat,
      so two correct solves end up to 2e-3 apart there at costs equal to 1e-9
      (as two CPU runs with different radii do, tests/test_solver_gpu.py::
      test_ill_conditioned_rpc_reaches_same_cost); mid-solve costs are not
      comparable either (a rounding change moves the truncated CG's stopping
      point and with it the LM path)."""
    R = rig.make_rig(num_sensors=3, num_ref=40, num_points=3000, obs_per_point=6, seed=13)
    # reference poses fixed: a unique minimum (no gauge directions)
    P = rig.build_problem(R, rig.FloatFlags(camera_poses_to_float=()))
    tol = dict(function_tolerance=1e-16, gradient_tolerance=1e-16, parameter_tolerance=1e-12)
    sysm = _exact_step_system(P)
    conv = []
    # "0": W z formed by pass A (MVBA_CG_DZ=passa); "update": the default (W z
    # from the update's frame blocks, the fused CG step at this size);
    # "nofuse": the same without the fused step; "1": the direction kernel
    for form in ("0", "update", "nofuse", "1"):
        monkeypatch.setenv("MVBA_CG_DIR_KERNEL", "1" if form == "1" else "0")
        monkeypatch.setenv("MVBA_CG_DZ", "passa" if form == "0" else "update")
        monkeypatch.setenv("MVBA_CG_FUSE", "0" if form == "nofuse" else "1")
        with Evaluator(P) as ev:
            ev.set_params()
            s = ev.solve(max_num_iterations=1, eta=1e-14, max_linear_solver_iterations=4000, use_loss=1,
                         robust_threshold=3.0, **tol)
            x = ev.get_params()
        assert s["num_linear_iterations"] > 10, s["num_linear_iterations"]
        _check_against_exact_step(sysm, x, f"form {form} ({s['num_linear_iterations']} CG iterations)")
        with Evaluator(P) as ev:
            ev.set_params()
            s = ev.solve(max_num_iterations=200, use_loss=1, robust_threshold=3.0, **tol)
            conv.append(s)
    sa = conv[0]
    for sb in conv:
        assert sb["termination_type"] == 0, sb["message"]
        assert np.isclose(sa["final_cost"], sb["final_cost"], rtol=1e-9), (sa["final_cost"], sb["final_cost"])


@pytest.mark.gpu
@pytest.mark.parametrize("exchange", ["none", "rccl"])
def test_atomic_exact_step_through_resets(exchange):
    """Atomic (non-deterministic) sums, CG to eta = 1e-14: dozens of
    iterations and several of Ceres' residual resets (r = b - A x every 10th
    iteration, a product in line), on one rank and through a one-rank RCCL
    communicator (fold-mode tail, the exchanged p.q, graphs with the
    all-reduce inside): the step against the CPU's exact step of the same
    system. (A side-stream form of the reset product measured slower,
    profiles/r06/r06l/.)"""
    import torch

    # reference poses fixed: a unique minimum (test_point_solve_forms_agree)
    R = rig.make_rig(num_sensors=3, num_ref=10, num_points=400, obs_per_point=4, seed=11)
    P = rig.build_problem(R, rig.FloatFlags(camera_poses_to_float=()))
    sysm = _exact_step_system(P)
    st = torch.cuda.Stream()
    comm = None
    if exchange == "rccl":
        from multiview_amd.dist import Comm

        comm = Comm.rccl_world1(0)
    try:
        n_det = 0
        for det in (1, 0):
            # the atomic run's CG runs at least the deterministic run's count:
            # at eta = 1e-14 the q-criterion fires at rounding stagnation, whose
            # iteration moves with the order of the atomic sums (tests/test_mesh.py)
            with Evaluator(P) as ev:
                ev.set_params()
                s = ev.solve(max_num_iterations=1, eta=1e-14, max_linear_solver_iterations=2000,
                             min_linear_solver_iterations=n_det, use_loss=1, robust_threshold=3.0,
                             deterministic=det, function_tolerance=1e-16, gradient_tolerance=1e-16,
                             parameter_tolerance=1e-16, comm=comm, stream=st.cuda_stream)
                x = ev.get_params()
            n_det = s["num_linear_iterations"]
    finally:
        if comm is not None:
            comm.close()
    assert s["num_linear_iterations"] > 20, s["num_linear_iterations"]
    assert s["final_cost"] < s["initial_cost"]
    _check_against_exact_step(sysm, x, f"atomic {exchange} ({s['num_linear_iterations']} CG iterations)")
