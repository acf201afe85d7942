"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Tolerances (DESIGN.md "Parity"):
  residuals        |r_gpu - r_oracle| <= 1e-9 * max(|pixel|, 1)
  Jacobian         |J_gpu - J_exact| <= 1e-9 * max(column max, 1e-12)   (exact = oracle dual numbers)
  vs reference FD  |J_gpu - J_numdiff| <= central-difference rounding bound (fd_bound)
"""
import zlib

import numpy as np
import pytest

from conftest import case_problem, fd_bound, golden_cases, golden_jacobian_row
from multiview_amd import _lib, rig
from multiview_amd.evaluator import Evaluator

pytestmark = pytest.mark.gpu

MODEL_SETS = {
    "none": ["none"] * 3,
    "fov": ["fov"] * 3,
    "radtan": ["radtan"] * 3,
    "radtan4": ["radtan4"] * 3,
    "rpc1": ["rpc1"] * 3,
    "rpc2": ["rpc2"] * 3,
    "rpc3": ["rpc3"] * 3,
    "mixed": ["radtan", "rpc2", "fov", "none"],
}


def _check(P, ev, oracle, apply_loss=False, numdiff=True):
    cost_g, r_g, J_g = ev.evaluate(jacobian=True, apply_loss=apply_loss)
    cost_o, r_o, J_o = oracle.evaluate(P, oracle.ANALYTIC, apply_loss=apply_loss)
    pix = np.maximum(np.abs(P.residual_meas + r_o).max(axis=1), 1.0)
    assert np.all(np.abs(r_g - r_o) <= 1e-9 * pix[:, None]), np.abs(r_g - r_o).max()
    assert np.isclose(cost_g, cost_o, rtol=1e-10)
    colmax = np.maximum(np.abs(J_o).max(axis=0), 1e-12)
    err = np.abs(J_g - J_o) / colmax
    assert err.max() <= 1e-9, (np.unravel_index(np.argmax(err), err.shape), err.max())
    # constant blocks stay zero (Ceres passes NULL jacobians for them)
    assert np.all((J_o == 0) | (J_g != 0) | (np.abs(J_o) < 1e-12 * colmax))
    if numdiff and not apply_loss:
        _, _, J_n = oracle.evaluate(P, oracle.NUMDIFF)
        assert np.all(np.abs(J_g - J_n) <= fd_bound(P, J_o, r_o))


@pytest.mark.parametrize("name", list(MODEL_SETS))
def test_parity_small_rig(oracle, name):
    models = MODEL_SETS[name]
    R = rig.make_rig(num_sensors=len(models), num_ref=24, num_points=300, obs_per_point=5,
                     models=models, seed=zlib.crc32(name.encode()) % 1000)
    P = rig.build_problem(R)
    with Evaluator(P) as ev:
        ev.set_params()
        _check(P, ev, oracle)


def test_parity_c1_full(oracle):
    """BASELINE config c1 (configs[0]) whole: 3-sensor rig, 1k landmarks /
    ~5k observations, pinhole without distortion, every block floating;
    residuals and Jacobian against the oracle's exact derivative, and against
    the reference's central differences within the FD bound."""
    R = rig.make_rig(**rig.CONFIGS["c1"])
    P = rig.build_problem(R)
    assert P.num_residuals > 4500 and set(P.camera_dist_size.tolist()) == {0}
    with Evaluator(P) as ev:
        ev.set_params()
        _check(P, ev, oracle)
        _check(P, ev, oracle, apply_loss=True)


def test_parity_no_rig(oracle):
    R = rig.make_rig(num_sensors=3, num_ref=20, num_points=300, obs_per_point=5, seed=77)
    P = rig.build_problem(R, rig.FloatFlags(no_rig=True, camera_poses_to_float=("ref_cam", "cam1", "cam2"),
                                            float_timestamp_offsets=False))
    with Evaluator(P) as ev:
        ev.set_params()
        _check(P, ev, oracle)


@pytest.mark.parametrize("flags", [
    rig.FloatFlags(camera_poses_to_float=(), rig_transforms_to_float=(), intrinsics_to_float=(),
                   float_timestamp_offsets=False),
    rig.FloatFlags(camera_poses_to_float=("ref_cam",), rig_transforms_to_float=("cam2",),
                   intrinsics_to_float=("distortion",), float_timestamp_offsets=True),
])
def test_parity_constant_blocks(oracle, flags):
    R = rig.make_rig(num_sensors=3, num_ref=20, num_points=300, obs_per_point=5, seed=78)
    P = rig.build_problem(R, flags)
    with Evaluator(P) as ev:
        ev.set_params()
        _check(P, ev, oracle)


def test_parity_cauchy_loss(oracle):
    R = rig.make_rig(num_sensors=3, num_ref=20, num_points=300, obs_per_point=5, seed=79, noise_px=4.0)
    P = rig.build_problem(R)
    with Evaluator(P) as ev:
        ev.set_params()
        _check(P, ev, oracle, apply_loss=True)


def test_device_loss_flag_matches_host_corrector(oracle):
    import torch

    R = rig.make_rig(num_sensors=3, num_ref=20, num_points=300, obs_per_point=5, seed=80, noise_px=4.0)
    P = rig.build_problem(R)
    with Evaluator(P) as ev:
        ev.set_params()
        ld = ev.ld
        res = torch.zeros((2, ld), dtype=torch.float64, device="cuda")
        jac = torch.zeros((ev.stride, ld), dtype=torch.float64, device="cuda")
        ev.evaluate_device(jacobian=True, apply_loss=True, robust_threshold=3.0, residuals=res, jac=jac, ld=ld)
        ev.sync()
        order = ev.order()
        valid = order >= 0
        assert valid.sum() == ev.num_residuals
        assert np.array_equal(np.sort(order[valid]), np.arange(ev.num_residuals))
        _, r_o, J_o = oracle.evaluate(P, oracle.ANALYTIC, apply_loss=True)
        r_d = res.cpu().numpy()[:, :ev.num_slots].T[valid]
        J_d = jac.cpu().numpy()[:, :ev.num_slots].T[valid]
        assert np.abs(r_d - r_o[order[valid]]).max() <= 1e-9 * 1024
        colmax = np.maximum(np.abs(J_o).max(axis=0), 1e-12)
        assert (np.abs(J_d - J_o[order[valid]]) / colmax).max() <= 1e-9


CASES = golden_cases()


def test_golden_vectors_on_gpu():
    for case in CASES:
        P = case_problem(case)
        with Evaluator(P) as ev:
            ev.set_params()
            _, r, J = ev.evaluate(jacobian=True)
        scale = max(1.0, abs(case["meas"][0]), abs(case["meas"][1]))
        assert np.abs(r[0] - np.array(case["residual"])).max() <= 1e-9 * scale, case["kind"]
        Jg = golden_jacobian_row(case, J.shape[1])
        tol = 1e-9 * np.maximum(np.abs(Jg), np.abs(Jg).max())
        assert np.all(np.abs(J[0] - Jg) <= np.maximum(tol, 1e-12)), (case["model"], case["kind"])


def test_alpha_out_of_range_reported():
    R = rig.make_rig(num_sensors=2, num_ref=8, num_points=50, obs_per_point=4, seed=81)
    P = rig.build_problem(R)
    # push sensor 1's offset outside its bracket: alpha < 0 (rig_calibrator.cc:346)
    b = P.residual_blocks[P.residual_camera == 1][0, 4]
    P.params[P.block_offset[b]] = 0.6
    with Evaluator(P) as ev:
        ev.set_params()
        with pytest.raises(_lib.MvbaError) as e:
            ev.evaluate(jacobian=False)
        assert e.value.status == _lib.MVBA_E_ALPHA_RANGE
        assert "Out of bounds in interpolation" in e.value.message


def test_bad_distortion_size_rejected():
    R = rig.make_rig(num_sensors=2, num_ref=8, num_points=50, obs_per_point=4, seed=82)
    P = rig.build_problem(R)
    P.camera_dist_size[:] = 6
    with pytest.raises(_lib.MvbaError) as e:
        Evaluator(P)
    assert e.value.status == _lib.MVBA_E_BAD_DISTORTION


def test_full_size_c2_properties(oracle):
    """BASELINE config c2 (1M observations): determinism, residual-only vs
    residual+Jacobian agreement, and a 4000-residual random sample vs the oracle."""
    import torch

    R = rig.make_rig(**rig.CONFIGS["c2"])
    P = rig.build_problem(R)
    with Evaluator(P) as ev:
        ev.set_params()
        n, S, ld = ev.num_residuals, ev.num_slots, ev.ld
        r1 = torch.empty((2, ld), dtype=torch.float64, device="cuda")
        j1 = torch.empty((ev.stride, ld), dtype=torch.float64, device="cuda")
        r2 = torch.empty_like(r1)
        j2 = torch.empty_like(j1)
        r3 = torch.empty_like(r1)
        ev.evaluate_device(True, residuals=r1, jac=j1, ld=ld)
        ev.evaluate_device(True, residuals=r2, jac=j2, ld=ld)
        ev.evaluate_device(False, residuals=r3, jac=None, ld=ld)
        ev.sync()
        order = ev.order()
        valid = torch.from_numpy(order >= 0).cuda()
        assert torch.equal(r1[:, :S][:, valid], r2[:, :S][:, valid])
        assert torch.equal(r1[:, :S][:, valid], r3[:, :S][:, valid])
        assert np.array_equal(np.sort(order[order >= 0]), np.arange(n))
        assert S <= n + 32 * ev.num_frames + 32  # frame ranges start on 32-slot boundaries
        rng = np.random.default_rng(5)
        slots = np.nonzero(order >= 0)[0]
        pos = np.sort(rng.choice(slots, 4000, replace=False))
        idx = order[pos]
        sub = P.subset(idx)
        _, r_o, J_o = oracle.evaluate(sub, oracle.ANALYTIC)
        J1 = j1[:, :S].cpu().numpy()
        r_g = r1[:, :S].cpu().numpy()[:, pos].T
        J_g = J1[:, pos].T
        pix = np.maximum(np.abs(sub.residual_meas + r_o).max(axis=1), 1.0)
        assert np.all(np.abs(r_g - r_o) <= 1e-9 * pix[:, None])
        colmax = np.maximum(np.abs(J_o).max(axis=0), 1e-12)
        written = J_o != 0
        assert (np.abs(J_g - J_o)[written] / np.broadcast_to(colmax, J_o.shape)[written]).max() <= 1e-9
