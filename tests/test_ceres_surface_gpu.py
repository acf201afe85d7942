"""GPU test of the header-only Ceres adapter (include/mvba/ceres_surface.h),
driven the way Ceres drives a CostFunction (tests/cpp/test_ceres_surface.cpp)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from multiview_amd import rig

pytestmark = pytest.mark.gpu

BIN = os.path.join(ROOT, "tests", "cpp", "test_ceres_surface")


def _write(fh, arr, dtype):
    a = np.ascontiguousarray(arr, dtype=dtype).reshape(-1)
    fh.write(np.int64(a.size).tobytes())
    fh.write(a.tobytes())


def _read(fh, dtype):
    n = int(np.frombuffer(fh.read(8), dtype=np.int64)[0])
    return np.frombuffer(fh.read(n * np.dtype(dtype).itemsize), dtype=dtype)


def test_ceres_adapter(tmp_path, oracle):
    if not os.path.exists(BIN):
        subprocess.run(["make", "-s", "-C", os.path.dirname(BIN)], check=True)
    run_adapter_case(BIN, tmp_path, oracle)


def run_adapter_case(binary, tmp_path, oracle, env=None):
    """Drive the adapter binary on a dumped problem and check every case;
    returns the binary's stderr (the sanitizer build checks it is clean)."""
    from test_mesh import _oracle_mesh_xyz

    # sphere-surface scene: depth, depth-mesh (BracketedDepthMeshError), mesh_tri
    # and tri blocks beside the reprojection blocks
    R = rig.make_rig(num_sensors=3, num_ref=30, num_points=300, obs_per_point=5,
                     models=["radtan", "rpc1", "fov"], seed=31, depth_sensors=(2,), affine_depth=False,
                     surface="sphere")
    F = rig.FloatFlags(depth_tri_weight=10.0, depth_to_image_transforms_to_float=("cam2",), float_scale=True,
                       tri_weight=0.5, tri_robust_threshold=0.1, depth_mesh_weight=5.0, mesh_tri_weight=2.0)
    mxyz = _oracle_mesh_xyz(R)
    P = rig.build_problem(R, F, mesh_xyz=mxyz)
    assert P.num_depth_residuals > 0 and P.num_xyz_residuals > 0 and (P.depth_blocks[:, 5] == -1).any()
    params2 = P.params.copy()
    params2 += np.random.default_rng(1).normal(0, 1e-4, params2.shape) * (P.params != 0)
    src = tmp_path / "prob.bin"
    with open(src, "wb") as fh:
        _write(fh, P.block_size, np.int32)
        _write(fh, P.block_offset, np.int64)
        _write(fh, P.params, np.float64)
        _write(fh, P.camera_dist_size, np.int32)
        _write(fh, P.camera_half_size, np.float64)
        _write(fh, P.residual_blocks, np.int32)
        _write(fh, P.residual_camera, np.int32)
        _write(fh, P.residual_meas, np.float64)
        _write(fh, P.residual_stamps, np.float64)
        _write(fh, params2, np.float64)
        _write(fh, P.depth_blocks, np.int32)
        _write(fh, P.block_size[P.depth_blocks[:, 3]], np.int32)
        _write(fh, P.depth_meas, np.float64)
        _write(fh, P.depth_weight, np.float64)
        _write(fh, P.depth_stamps, np.float64)
        _write(fh, P.xyz_block, np.int32)
        _write(fh, P.xyz_ref, np.float64)
        _write(fh, P.xyz_weight, np.float64)
        _write(fh, P.depth_mesh_xyz, np.float64)
    out = tmp_path / "out.bin"
    p = subprocess.run([binary, str(src), str(out)], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    n = P.num_residuals
    stride = P.jacobian_stride()
    with open(out, "rb") as fh:
        R0, J0 = _read(fh, np.float64), _read(fh, np.float64)
        J1 = _read(fh, np.float64)
        R2, J2 = _read(fh, np.float64), _read(fh, np.float64)
        R4, J4 = _read(fh, np.float64), _read(fh, np.float64)
        R5, J5 = _read(fh, np.float64), _read(fh, np.float64)
        R6, J6 = _read(fh, np.float64), _read(fh, np.float64)
        J6b = _read(fh, np.float64)
        sizes6 = _read(fh, np.int64)
        RD, JD, RX, JX = (_read(fh, np.float64) for _ in range(4))
        R8, J8, RD8, JD8, RX8, JX8 = (_read(fh, np.float64) for _ in range(6))
        flags = _read(fh, np.int32)
    # full Jacobians: the adapter evaluates every block (all free)
    Pf = rig.build_problem(R, F, mesh_xyz=mxyz)
    Pf.block_constant[:] = 0
    _, r_o, J_o = oracle.evaluate(Pf, oracle.ANALYTIC)
    P2 = rig.build_problem(R, F, mesh_xyz=mxyz)
    P2.block_constant[:] = 0
    P2.params = params2
    _, r_o2, J_o2 = oracle.evaluate(P2, oracle.ANALYTIC)

    def close(r, J, r_ref, J_ref):
        colmax = np.maximum(np.abs(J_ref).max(axis=0), 1e-12)
        return (np.abs(r.reshape(n, 2) - r_ref).max() <= 1e-9 * 1024 and
                (np.abs(J.reshape(n, stride) - J_ref) / colmax).max() <= 1e-9)

    assert flags[0] == 1 and close(R0, J0, r_o, J_o)
    J1 = J1.reshape(n, stride)
    assert flags[1] == 1
    assert np.all(J1[:, 14:28] == 0) and np.all(J1[:, 56:] == 0)  # NULL blocks untouched
    assert np.allclose(J1[:, :14], J_o[:, :14], rtol=0, atol=1e-9 * np.abs(J_o).max())
    assert flags[2] == 1 and flags[3] == 1 and close(R2, J2, r_o2, J_o2)  # one GPU pass
    assert flags[4] == 0  # point not in user memory -> Evaluate() false
    assert flags[5] == 1 and flags[6] == 1 and close(R4, J4, r_o, J_o)
    assert flags[7] == 0 and close(R5, J5, r_o2, J_o2)
    # (6) packed transfer: end and distortion never asked -> not transferred
    assert flags[8] == 1 and flags[9] == 1
    K = P.camera_dist_size[P.residual_camera]
    width = np.array([7, 7, 7, 3, 1, 1, 2, 0])[None, :].repeat(n, 0)
    width[:, 7] = K
    assert sizes6[0] == 2 * int(width.sum())                    # first pass: every block
    # afterwards only blocks Ceres asked for at some position (a world_to_ref block
    # is the end of one bracket and the beginning of the next)
    asked = np.zeros(len(P.block_size), bool)
    for b in (0, 2, 3, 4, 5, 6):
        asked[P.residual_blocks[:, b]] = True
    assert sizes6[1] == 2 * int((width * asked[P.residual_blocks]).sum()) < sizes6[0]
    J6 = J6.reshape(n, stride)
    mask = np.ones(stride, bool)
    mask[14:28] = False
    mask[56:] = False
    assert np.all(J6[:, ~mask] == 0) and close(R6, np.where(mask, J6, J_o), r_o, J_o)
    assert flags[10] == 1 and flags[11] == 1 and close(R6, J6b, r_o, J_o)  # one extension pass
    assert sizes6[2] == sizes6[0]
    # (7) depth + xyz blocks from the same batch, one GPU pass
    assert flags[12] == 1 and flags[13] == 1
    _, rd_o, Jd_o = oracle.evaluate_depth(Pf, oracle.ANALYTIC)
    nd = P.num_depth_residuals
    dscale = max(np.abs(rd_o).max(), 1.0)
    assert np.abs(RD.reshape(nd, 3) - rd_o).max() <= 1e-9 * dscale
    JD = JD.reshape(nd, -1)
    assert (np.abs(JD - Jd_o) / np.maximum(np.abs(Jd_o).max(axis=0), 1e-12)).max() <= 1e-9
    X = np.stack([Pf.block_values(int(b)) for b in P.xyz_block])
    w = P.xyz_weight[:, None]
    assert np.allclose(RX.reshape(-1, 3), w * (X - P.xyz_ref), rtol=0, atol=1e-12)
    assert np.allclose(JX.reshape(-1, 3, 3), P.xyz_weight[:, None, None] * np.eye(3), rtol=0, atol=0)
    # (8) the reference's own Create / AddResidualBlock statements (only the
    # namespace qualifier changed): blocks read back from the ceres::Problem,
    # same residuals and Jacobians as the explicit-pointer batch and the oracle
    nx = P.num_xyz_residuals
    assert flags[14] == 1, "case 8: an Evaluate() failed"
    assert flags[15] == 2  # the lazy pass, then the callback's pass
    assert flags[16] == n + nd + nx
    assert flags[17] == 1  # a static factory without a problem-bound batch throws
    assert close(R8, J8, r_o, J_o)
    assert np.array_equal(R8, R0) and np.array_equal(J8, J0)
    assert np.array_equal(RD8, RD) and np.array_equal(JD8, JD.ravel())
    assert np.array_equal(RX8, RX) and np.array_equal(JX8, JX)
    return p.stderr
