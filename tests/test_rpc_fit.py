"""RPC lens-model fits: mvba_rpc_fit against the oracle's
restatement (oracle/rpc_fit_reference.py) of genUndistDistPairs, fitRpcDist,
fitRpcUndist and evalRpcDistUndist (rpc_distortion.cc:519-737).

The oracle is pinned by exact recovery: when the camera's distortion is itself
an RPC model of the fitted degree, the least-squares minimum has zero residual
and both fits must reproduce the camera to 1e-8 px. GPU parity compares the
fitted models' outputs on the samples (tolerance 1e-6 px; the two LM runs take
different paths to the same minimum), the sample counts (exact) and bounding
boxes (1e-12)."""
import numpy as np
import pytest

from multiview_amd import _lib, rig
from oracle import rpc_fit_reference as rf

RADTAN_CAM = dict(focal=600.0, center=(515.0, 382.0), dist=np.array(rig.RADTAN), image_size=(1024, 768),
                  crop_size=(1000, 740), undist_size=(1100, 800))


def _rpc_cam(deg, seed=5):
    c = rig.default_coeffs(f"rpc{deg}", np.random.default_rng(seed))
    return dict(focal=600.0, center=(512.0, 384.0), dist=c, image_size=(1024, 768), crop_size=(1024, 768),
                undist_size=(1024, 768)), c[:c.size // 2]


def test_identity_and_increment_layout():
    p = np.random.default_rng(0).normal(size=(50, 2)) * 100
    c = rf.identity(1)
    assert np.allclose(rf.compute_rpc(p, c), p)
    for _ in range(3):  # added zero terms leave the model unchanged
        c = rf.increment_degree(c)
        assert np.allclose(rf.compute_rpc(p, c), p)
    assert c.size == 2 * 5 * 6 - 2


def test_oracle_recovers_an_rpc_camera_exactly():
    cam, dist = _rpc_cam(2)
    c, u = rf.fit_rpc_dist(cam, 2, 60)
    assert np.abs(rf.compute_rpc(u, c) - rf.compute_rpc(u, dist)).max() < 1e-8


def test_bad_distortion_rejected_before_device():
    from multiview_amd.rpc_fit import fit_rpc_distortion

    cam = dict(RADTAN_CAM, dist=np.zeros(7))
    with pytest.raises(_lib.MvbaError) as e:
        fit_rpc_distortion(cam, 2)
    assert e.value.status == _lib.MVBA_E_BAD_DISTORTION


@pytest.mark.gpu
@pytest.mark.parametrize("degree", [1, 2, 3])
def test_fit_distortion_matches_oracle(degree):
    from multiview_amd.rpc_fit import fit_rpc_distortion

    S = 120
    c_g, rep = fit_rpc_distortion(RADTAN_CAM, degree, num_samples=S)
    c_o, u = rf.fit_rpc_dist(RADTAN_CAM, degree, S)
    assert rep["num_samples_used"] == len(u)
    u_all, d_all = rf.pairs(RADTAN_CAM, S)
    assert np.allclose(rep["undist_box"], [*u_all.min(0), *u_all.max(0)], rtol=0, atol=1e-12)
    assert np.allclose(rep["dist_box"], [*d_all.min(0), *d_all.max(0)], rtol=0, atol=1e-9)
    assert np.abs(rf.compute_rpc(u, c_g) - rf.compute_rpc(u, c_o)).max() < 1e-6
    assert _lib.FAILURE not in rep["termination"]


@pytest.mark.gpu
def test_fit_distortion_recovers_rpc_camera():
    from multiview_amd.rpc_fit import fit_rpc_distortion

    cam, dist = _rpc_cam(2)
    c_g, rep = fit_rpc_distortion(cam, 2, num_samples=80)
    u, _ = rf.pairs(cam, 80)
    assert np.abs(rf.compute_rpc(u, c_g) - rf.compute_rpc(u, dist)).max() < 1e-8


@pytest.mark.gpu
@pytest.mark.parametrize("deg", [2, 3])
def test_fit_undistortion_matches_oracle(deg):
    """updateRpcUndistortion: the camera's RPC distortion half fixed, the
    undistortion half refit; evalRpcDistUndist's max round-trip error."""
    from multiview_amd.rpc_fit import fit_rpc_undistortion

    cam, dist = _rpc_cam(deg, seed=11)
    S = 150
    c_g, rep = fit_rpc_undistortion(cam, dist, num_samples=S)
    c_o, u, dc, err = rf.fit_rpc_undist(cam, dist, S)
    assert rep["num_samples_used"] == len(u)
    assert np.abs(rf.compute_rpc(dc, c_g) - rf.compute_rpc(dc, c_o)).max() < 1e-6
    assert abs(rep["max_dist_undist_error"] - err) < 1e-6
    assert rep["max_dist_undist_error"] < 1e-3  # the refit inverts the distortion
