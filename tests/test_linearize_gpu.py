"""GPU parity of the normal-equation kernels (K2: camera-side fp64-MFMA Gram +
expand, point-side kernel) against J^T r and J_b^T J_b built from the oracle's
exact Jacobian. Tolerance: 1e-9 of each block's largest entry."""
import zlib

import numpy as np
import pytest

from multiview_amd import rig
from multiview_amd.evaluator import Evaluator
from oracle.normal_equations import normal_equations_reference

pytestmark = pytest.mark.gpu

MODEL_SETS = {
    "none": ["none"] * 3,
    "fov": ["fov"] * 3,
    "radtan": ["radtan"] * 3,
    "radtan4": ["radtan4", "radtan", "radtan"],
    "rpc1": ["rpc1"] * 3,
    "rpc2": ["rpc2"] * 3,
    "rpc3": ["rpc3"] * 3,
    "rpc4": ["rpc4", "radtan"],
    "rpc5": ["rpc5", "fov"],
    "rpc6": ["rpc6", "none"],
    "mixed": ["radtan", "rpc2", "fov", "none"],
    "mixed_high": ["rpc4", "rpc6", "radtan"],
}


def _blockwise_close(got, ref, offs, sizes, tol=1e-9):
    for o, n in zip(offs, sizes):
        a, b = got[o:o + n], ref[o:o + n]
        scale = max(np.abs(b).max(), 1e-300)
        assert np.abs(a - b).max() <= tol * scale, (o, n, np.abs(a - b).max(), scale)


def _run(P, oracle, apply_loss):
    import torch

    with Evaluator(P) as ev:
        ev.set_params()
        L = ev.lin_layout()
        assert L["supported"]
        dev = "cuda"
        cg = torch.zeros(L["cam_grad_size"], dtype=torch.float64, device=dev)
        ch = torch.zeros(L["cam_hess_size"], dtype=torch.float64, device=dev)
        pg = torch.zeros(3 * L["num_points"], dtype=torch.float64, device=dev)
        ph = torch.zeros(6 * L["num_points"], dtype=torch.float64, device=dev)
        cost = torch.zeros(1, dtype=torch.float64, device=dev)
        ev.linearize_device(cg, ch, pg, ph, cost, apply_loss=apply_loss, robust_threshold=3.0)
        ev.sync()
        c_o, r_o, J_o = oracle.evaluate(P, oracle.ANALYTIC, apply_loss=apply_loss, robust_threshold=3.0)
        g_ref, h_ref, pg_ref, ph_ref = normal_equations_reference(P, r_o, J_o, L)
        sizes = P.block_size[L["cam_block_ids"]]
        _blockwise_close(cg.cpu().numpy(), g_ref, L["cam_goff"], sizes)
        _blockwise_close(ch.cpu().numpy(), h_ref, L["cam_hoff"], sizes * sizes)
        npt = L["num_points"]
        _blockwise_close(pg.cpu().numpy(), pg_ref, 3 * np.arange(npt), [3] * npt)
        _blockwise_close(ph.cpu().numpy(), ph_ref, 6 * np.arange(npt), [6] * npt)
        assert np.isclose(cost.item(), c_o, rtol=1e-11)


@pytest.mark.parametrize("name", list(MODEL_SETS))
@pytest.mark.parametrize("apply_loss", [False, True])
def test_linearize_parity(oracle, name, apply_loss):
    models = MODEL_SETS[name]
    R = rig.make_rig(num_sensors=len(models), num_ref=20, num_points=300, obs_per_point=6,
                     models=models, seed=zlib.crc32(name.encode()) % 997, noise_px=2.0)
    P = rig.build_problem(R)
    _run(P, oracle, apply_loss)


def test_linearize_constant_blocks_and_no_rig(oracle):
    R = rig.make_rig(num_sensors=3, num_ref=16, num_points=250, obs_per_point=5, seed=91)
    P = rig.build_problem(R, rig.FloatFlags(camera_poses_to_float=("ref_cam",), rig_transforms_to_float=("cam2",),
                                            intrinsics_to_float=("distortion",), float_timestamp_offsets=False))
    _run(P, oracle, True)
    P2 = rig.build_problem(R, rig.FloatFlags(no_rig=True, camera_poses_to_float=("ref_cam", "cam1"),
                                             float_timestamp_offsets=False))
    _run(P2, oracle, False)


def test_linearize_long_frames_rpc_wide(oracle):
    # a frame split into several parts (> kPartSegs segments) with the wide-Gram
    # (rows straight into LDS) path of RPC degree 2
    R = rig.make_rig(num_sensors=2, num_ref=4, num_points=5000, obs_per_point=3, models=["rpc2", "radtan"], seed=94,
                     window=2)
    P = rig.build_problem(R)
    counts = np.bincount(R.obs_cid)
    assert counts.max() > 16 * 64
    _run(P, oracle, True)


def test_linearize_long_frames(oracle):
    # frames with more than kChunkSegs * 64 observations: several chunks per frame
    R = rig.make_rig(num_sensors=2, num_ref=6, num_points=1500, obs_per_point=4, seed=92, window=3)
    P = rig.build_problem(R)
    counts = np.bincount(R.obs_cid)
    assert counts.max() > 256
    _run(P, oracle, True)
