"""The one-launch forms of mvba_evaluate_device against the two-launch form.

mvba_evaluate_device runs one launch for a one-group problem: k_eval_local by
default (each block computes the K0 record of each of its frames once in LDS,
its waves of one frame sharing it; npts 120: one segment per frame, 2500:
~5, frames spanning blocks) or, forced by
MVBA_EVAL_MODE=fused, k_eval (K0 blocks hand the records to the K1 waves of the
same grid). Both must write bit-identical planes to the two-launch form (the
prep kernel, MVBA_EVAL_PREP_ONLY, then K1 with MVBA_EVAL_SKIP_PREP: the same
arithmetic), and the frame records and landmark records they leave behind must
serve a later SKIP_PREP evaluation (what the solver and the bench's instrumented
steps rely on)."""
import numpy as np
import pytest

from multiview_amd import _lib, rig
from multiview_amd.evaluator import Evaluator


@pytest.mark.gpu
@pytest.mark.parametrize("npts", [120, 2500])
@pytest.mark.parametrize("form", ["k_eval_local", "k_eval"])
@pytest.mark.parametrize("jacobian", [True, False])
def test_one_launch_evaluation_matches_two_launches(monkeypatch, npts, form, jacobian):
    import torch

    R = rig.make_rig(num_sensors=3, num_ref=10, num_points=npts, obs_per_point=4, seed=5)
    P = rig.build_problem(R)
    if form == "k_eval":
        monkeypatch.setenv("MVBA_EVAL_MODE", "fused")
    with Evaluator(P) as ev:
        ev.set_params()
        obs = np.bincount(R.obs_cid)
        assert ev.num_frames == (obs > 0).sum()
        assert ev.eval_form() == (_lib.FORM_FUSED if form == "k_eval" else _lib.FORM_LOCAL)
        ld = ev.ld
        outs = []
        # before every form the frame and landmark records are made stale: a
        # full prep at slightly different parameters, then the real ones set,
        # so a record entry the form under test does not rewrite shows up
        stale = P.params * (1.0 + 1e-6) + 1e-9
        for phases in ([0], [_lib.EVAL_PREP_ONLY, _lib.EVAL_SKIP_PREP], [0, _lib.EVAL_SKIP_PREP]):
            ev.set_params(stale)
            ev.evaluate_device(jacobian, phase=_lib.EVAL_PREP_ONLY)
            ev.set_params()
            res = torch.full((2, ld), float("nan"), dtype=torch.float64, device="cuda")
            jac = torch.full((ev.stride, ld), float("nan"), dtype=torch.float64, device="cuda") if jacobian else None
            for ph in phases:
                ev.evaluate_device(jacobian, residuals=res, jac=jac, ld=ld, phase=ph)
            torch.cuda.synchronize()
            ev.sync()
            outs.append((res.cpu().numpy(), jac.cpu().numpy() if jacobian else None))
    for r, J in outs[1:]:
        np.testing.assert_array_equal(r, outs[0][0])
        if jacobian:
            np.testing.assert_array_equal(J, outs[0][1])
    # every observation's residual slot was written
    with Evaluator(P) as ev:
        order = ev.order()
    assert np.isfinite(outs[0][0][:, : order.size][:, order >= 0]).all()


@pytest.mark.gpu
def test_fused_wait_gives_up_with_an_error(monkeypatch):
    """k_eval's K1 waves wait for their frame's K0 block with a bounded poll.
    A wave that gives up raises error word [1], and mvba_sync_status reports
    MVBA_E_DEVICE_WAIT instead of handing back residuals built from a record
    that may be stale. MVBA_EVAL_POLL_LIMIT=0 makes every wave raise the error
    before its first poll (read per call; deterministic, whatever the dispatch
    timing); the next evaluation at the default limit is clean again."""
    import torch

    R = rig.make_rig(num_sensors=3, num_ref=10, num_points=2500, obs_per_point=4, seed=5)
    P = rig.build_problem(R)
    monkeypatch.setenv("MVBA_EVAL_MODE", "fused")  # k_local is the default form
    with Evaluator(P) as ev:
        ev.set_params()
        assert ev.eval_form() == _lib.FORM_FUSED
        ref = None
        for limit in ("0", None):
            if limit is None:
                monkeypatch.delenv("MVBA_EVAL_POLL_LIMIT", raising=False)
            else:
                monkeypatch.setenv("MVBA_EVAL_POLL_LIMIT", limit)
            res = torch.full((2, ev.ld), float("nan"), dtype=torch.float64, device="cuda")
            ev.evaluate_device(False, residuals=res, ld=ev.ld)
            torch.cuda.synchronize()
            if limit == "0":
                with pytest.raises(_lib.MvbaError) as e:
                    ev.sync()
                assert e.value.status == _lib.MVBA_E_DEVICE_WAIT
            else:
                ev.sync()
                ref = res.cpu().numpy()
        # the clean evaluation equals the two-launch form
        res2 = torch.full((2, ev.ld), float("nan"), dtype=torch.float64, device="cuda")
        ev.evaluate_device(False, residuals=res2, ld=ev.ld, phase=_lib.EVAL_PREP_ONLY)
        ev.evaluate_device(False, residuals=res2, ld=ev.ld, phase=_lib.EVAL_SKIP_PREP)
        torch.cuda.synchronize()
        ev.sync()
        np.testing.assert_array_equal(res2.cpu().numpy(), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("npts,models", [(120, ["radtan", "radtan4", "radtan"]), (2500, ["rpc2"] * 3),
                                          (60, ["radtan", "fov", "radtan"])])
@pytest.mark.parametrize("mode", [None, "fused"])
def test_every_form_matches_the_oracle(oracle, monkeypatch, npts, models, mode):
    """The one-launch forms (k_eval_local, the default; k_eval with
    MVBA_EVAL_MODE=fused; the two-group problem runs split) and the two-launch
    form agree with the oracle
    per residual block on planes initialised to NaN: constant blocks differ
    between sensors (ref_cam poses float, cam1's rig transform floats), radtan
    K = 4 and 5 share a model group, fov and radtan are two groups."""
    import torch

    R = rig.make_rig(num_sensors=len(models), num_ref=10, num_points=npts, obs_per_point=4, models=models, seed=7)
    P = rig.build_problem(R, rig.FloatFlags(camera_poses_to_float=("ref_cam",), rig_transforms_to_float=("cam1",),
                                            intrinsics_to_float=("focal_length", "distortion")))
    _, r_o, J_o = oracle.evaluate(P, oracle.ANALYTIC)
    colmax = np.maximum(np.abs(J_o).max(axis=0), 1e-12)
    if mode:
        monkeypatch.setenv("MVBA_EVAL_MODE", mode)
    with Evaluator(P) as ev:
        ev.set_params()
        order = ev.order()
        valid = order >= 0
        for phases in ([0], [_lib.EVAL_PREP_ONLY, _lib.EVAL_SKIP_PREP]):
            res = torch.full((2, ev.ld), float("nan"), dtype=torch.float64, device="cuda")
            jac = torch.full((ev.stride, ev.ld), float("nan"), dtype=torch.float64, device="cuda")
            for ph in phases:
                ev.evaluate_device(True, residuals=res, jac=jac, ld=ev.ld, phase=ph)
            torch.cuda.synchronize()
            ev.sync()
            r = res.cpu().numpy()[:, : ev.num_slots][:, valid].T
            J = jac.cpu().numpy()[:, : ev.num_slots][:, valid].T
            idx = order[valid]
            pix = np.maximum(np.abs(P.residual_meas + r_o).max(axis=1), 1.0)[idx]
            assert np.all(np.abs(r - r_o[idx]) <= 1e-9 * pix[:, None])
            # the oracle's non-zero entries agree; where the oracle has a zero
            # (constant block of that residual) the plane holds zero or was not
            # written at all (NaN)
            Jo = J_o[idx]
            cm = np.broadcast_to(colmax, Jo.shape)
            live = Jo != 0
            assert np.all(np.abs(J[live] - Jo[live]) <= 1e-9 * cm[live])
            dead = ~live & np.isfinite(J)
            assert np.all(np.abs(J[dead]) <= 1e-9 * cm[dead])


@pytest.mark.gpu
def test_dense_frames_take_the_split_form(monkeypatch):
    """Past 24 segments (1,536 observations) per frame the default form is the
    split one (prep launch + K1: c4's ~39 segments per frame measured 12 %
    faster than k_eval_local, profiles/r05/r05w/), and it writes the same
    planes as the forced one-launch form."""
    import torch

    R = rig.make_rig(num_sensors=1, num_ref=4, num_points=3000, obs_per_point=3, seed=9)
    P = rig.build_problem(R)
    outs = []
    for mode in (None, "local"):
        if mode:
            monkeypatch.setenv("MVBA_EVAL_MODE", mode)
        with Evaluator(P) as ev:
            ev.set_params()
            assert ev.num_residuals > 24 * 64 * ev.num_frames
            assert ev.eval_form() == (_lib.FORM_LOCAL if mode else _lib.FORM_SPLIT)
            res = torch.full((2, ev.ld), float("nan"), dtype=torch.float64, device="cuda")
            jac = torch.full((ev.stride, ev.ld), float("nan"), dtype=torch.float64, device="cuda")
            ev.evaluate_device(True, residuals=res, jac=jac, ld=ev.ld)
            torch.cuda.synchronize()
            ev.sync()
            outs.append((res.cpu().numpy(), jac.cpu().numpy()))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
