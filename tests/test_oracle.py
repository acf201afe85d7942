"""CPU tests of the oracle restatement (no GPU): golden vectors, known answers,
structural zeros, the reference's error conditions and central differences."""
import numpy as np
import pytest

from conftest import case_problem, fd_bound, golden_cases, golden_jacobian_row
from multiview_amd import rig
from multiview_amd._lib import JAC_BASE
from multiview_amd.problem import ProblemBuilder

CASES = golden_cases()


@pytest.mark.parametrize("ci", range(len(CASES)), ids=[f"{c['model']}-{c['kind']}" for c in CASES])
def test_oracle_matches_mpmath_golden(oracle, ci):
    case = CASES[ci]
    P = case_problem(case)
    _, r, _ = oracle.evaluate(P, oracle.RESIDUAL)
    scale = max(1.0, abs(case["meas"][0]), abs(case["meas"][1]))
    # fp64 restatement vs 50-digit value: a few ulps of the pixel magnitude
    assert np.abs(r[0] - np.array(case["residual"])).max() <= 1e-12 * scale
    _, _, Ja = oracle.evaluate(P, oracle.ANALYTIC)
    Jg = golden_jacobian_row(case, Ja.shape[1])
    colmax = np.maximum(np.abs(Jg), 1e-300)
    err = np.abs(Ja[0] - Jg)
    # per column, normalised by max(|J|, pixel-scale/|x| cancellation floor)
    tol = 1e-9 * np.maximum(np.abs(Jg).max(), 1.0)
    assert (err <= np.maximum(1e-8 * colmax, tol)).all(), (np.argmax(err), err.max())


def test_numdiff_matches_analytic_within_fd_bound(oracle):
    R = rig.make_rig(**rig.CONFIGS["c1"])
    P = rig.build_problem(R)
    _, r, Jn = oracle.evaluate(P, oracle.NUMDIFF)
    _, _, Ja = oracle.evaluate(P, oracle.ANALYTIC)
    assert (np.abs(Jn - Ja) <= fd_bound(P, Ja, r)).all()


@pytest.mark.parametrize("model", ["rpc2", "rpc3", "fov"])
def test_numdiff_rpc_fd_error_is_exactly_rational(oracle, model):
    # The reference's FD error on RPC denominator columns is the rational factor
    # 1/(1-x^2); everything else within rounding/truncation.
    for seed in (1, 2):
        R = rig.make_rig(num_sensors=3, num_ref=12, num_points=120, obs_per_point=5,
                         models=[model] * 3, seed=seed)
        P = rig.build_problem(R)
        _, r, Jn = oracle.evaluate(P, oracle.NUMDIFF)
        _, _, Ja = oracle.evaluate(P, oracle.ANALYTIC)
        assert (np.abs(Jn - Ja) <= fd_bound(P, Ja, r)).all()


def _identity_problem(K, coeffs, X=(0.0, 0.0, 3.0), center=(515.0, 382.0), f=600.0):
    pb = ProblemBuilder()
    beg = pb.add_parameter_block([0, 0, 0, 0, 0, 0, 1])
    end = pb.add_parameter_block([0, 0, 0, 0, 0, 0, 1])
    r2c = pb.add_parameter_block([0, 0, 0, 0, 0, 0, 1])
    xyz = pb.add_parameter_block(X)
    off = pb.add_parameter_block([0.0])
    foc = pb.add_parameter_block([f])
    ctr = pb.add_parameter_block(center)
    dst = pb.add_parameter_block(coeffs if K else [0.0])
    if not K:
        pb.set_parameter_block_constant(dst)
    cam = pb.add_camera(K, (1024, 768))
    pb.add_residual_block((0.0, 0.0), 5.0, 5.0, 5.0, [beg, end, r2c, xyz, off, foc, ctr, dst], cam)
    return pb.build()


@pytest.mark.parametrize("K,coeffs", [(0, []), (4, [-0.2, 0.05, 1e-3, 2e-3]), (5, [-0.25, 0.07, 1e-3, -5e-4, 0.01]),
                                      (1, [0.9])])
def test_known_answer_axis_point_maps_to_center(oracle, K, coeffs):
    # identity pose, X on the optical axis: d = c (NONE / FOV / RADTAN)
    P = _identity_problem(K, coeffs)
    _, r, _ = oracle.evaluate(P, oracle.RESIDUAL)
    assert np.allclose(r[0], [515.0, 382.0], atol=1e-12)


@pytest.mark.parametrize("deg", [1, 2, 3])
def test_known_answer_rpc_identity(oracle, deg):
    # RPCLensDistortion::init_as_identity (rpc_distortion.cc:303-318): d = u + h
    n = 2 * (deg + 1) * (deg + 2) - 2
    nl = (deg + 1) * (deg + 2) // 2
    half = np.zeros(n)
    half[1] = 1.0
    half[nl + nl - 1 + 2] = 1.0
    P = _identity_problem(2 * n, np.concatenate([half, half]), X=(0.3, -0.2, 2.0))
    _, r, J = oracle.evaluate(P, oracle.ANALYTIC)
    u = 600.0 * np.array([0.3 / 2.0, -0.2 / 2.0])
    assert np.allclose(r[0], u + np.array([512.0, 384.0]), atol=1e-12)
    # structural zeros: optical centre and the undistortion half
    assert np.all(J[0, JAC_BASE[6]:JAC_BASE[6] + 4] == 0.0)
    K = 2 * n
    dist = J[0, JAC_BASE[7]:JAC_BASE[7] + 2 * K].reshape(2, K)
    assert np.all(dist[:, n:] == 0.0)


def test_structural_zero_columns(oracle):
    R = rig.make_rig(**rig.CONFIGS["c1"])
    P = rig.build_problem(R)
    _, _, J = oracle.evaluate(P, oracle.ANALYTIC)
    ref = P.residual_camera == 0
    # ref-type observations: end, ref_to_cam, offset are constant (blocks NULL) -> zero
    assert np.all(J[ref][:, JAC_BASE[1]:JAC_BASE[3]] == 0.0)
    assert np.all(J[ref][:, JAC_BASE[4]:JAC_BASE[4] + 2] == 0.0)
    # the q direction of every free quaternion block is a null direction
    for b in (0, 1, 2):
        for i in np.nonzero(~ref)[0][:200]:
            q = P.block_values(P.residual_blocks[i, b])[3:]
            blk = J[i, JAC_BASE[b]:JAC_BASE[b] + 14].reshape(2, 7)
            if np.any(blk):
                assert np.abs(blk[:, 3:] @ q).max() <= 1e-9 * np.abs(blk).max()


def test_alpha_out_of_range_is_fatal(oracle):
    P = _identity_problem(0, [])
    P.residual_stamps[0] = [10.0, 11.0, 12.5]  # alpha = 2.5 (rig_calibrator.cc:346)
    with pytest.raises(oracle.OracleError) as e:
        oracle.evaluate(P, oracle.RESIDUAL)
    assert e.value.status == 1


@pytest.mark.parametrize("K", [2, 3, 6, 7, 10, 21])
def test_irregular_distortion_size_rejected(oracle, K):
    P = _identity_problem(0, [])
    P.camera_dist_size[:] = K
    st, msg = oracle.validate(P)
    assert st == 3 and "irregular distortion" in msg


def test_block_sizes_rejected(oracle):
    P = _identity_problem(0, [])
    P.block_size[3] = 4  # xyz block of size 4
    st, msg = oracle.validate(P)
    assert st == 2 and "block sizes" in msg


def test_cauchy_corrector(oracle):
    R = rig.make_rig(**rig.CONFIGS["c1"])
    P = rig.build_problem(R)
    c0, r0, J0 = oracle.evaluate(P, oracle.ANALYTIC)
    c1, r1, J1 = oracle.evaluate(P, oracle.ANALYTIC, apply_loss=True, robust_threshold=3.0)
    s = (r0 ** 2).sum(axis=1)
    rho0 = 9.0 * np.log1p(s / 9.0)
    sr = np.sqrt(1.0 / (1.0 + s / 9.0))
    assert np.isclose(c1, 0.5 * rho0.sum(), rtol=1e-12)
    assert np.isclose(c0, 0.5 * s.sum(), rtol=1e-12)
    assert np.allclose(r1, r0 * sr[:, None], rtol=1e-14, atol=0)
    assert np.allclose(J1, J0 * sr[:, None], rtol=1e-14, atol=0)


def test_residual_stats_percentiles(oracle):
    # rig_calibrator.cc:774-786: index int(0.25*len) etc. of the sorted |r|
    vals = np.array([3.0, -1.0, 2.0, -5.0, 4.0, 0.5, -0.25])
    ids = np.zeros(vals.size, dtype=np.int32)
    out, cnt = oracle.residual_stats(vals, ids, 1)
    s = np.sort(np.abs(vals))
    n = len(s)
    assert cnt[0] == n
    assert np.allclose(out[0], [s[int(0.25 * n)], s[int(0.5 * n)], s[int(0.75 * n)], s[n - 1]])


# ------------------------------------------------------------ depth golden vectors
def _depth_golden():
    import json
    import os

    with open(os.path.join(os.path.dirname(__file__), "golden", "depth_error_golden.json")) as f:
        return json.load(f)["cases"]


DEPTH_CASES = _depth_golden()


@pytest.mark.parametrize("ci", range(len(DEPTH_CASES)))
def test_oracle_depth_matches_mpmath_golden(oracle, ci):
    """BracketedDepthError (rig_calibrator.cc:547-583): the oracle's restatement
    against the independent 50-digit mpmath one (tests/golden/make_golden_depth.py),
    rigid and affine depth_to_image, reference / interpolated / no-rig frames,
    scale != 1. Residuals 1e-12 relative, Jacobian 1e-8 of each block's largest entry."""
    import numpy as np

    c = DEPTH_CASES[ci]
    blocks = [np.array(b) for b in c["blocks"]]
    r, J = oracle.depth_error(blocks, np.zeros(7, np.uint8), c["weight"], c["meas"], *c["stamps"],
                              mode=oracle.ANALYTIC)
    rg = np.array(c["residual"])
    assert np.abs(r - rg).max() <= 1e-12 * max(np.abs(rg).max(), 1.0)
    off = 0
    for b, blk in enumerate(blocks):
        n = 3 * blk.size
        Jg = np.array(c["jacobian"][b])
        scale = max(np.abs(Jg).max(), 1e-300)
        assert np.abs(J[off:off + n] - Jg).max() <= 1e-8 * scale, (b, np.abs(J[off:off + n] - Jg).max() / scale)
        off += n


# ------------------------------------------------------- depth-mesh golden vectors
def _depth_mesh_golden():
    import json
    import os

    with open(os.path.join(os.path.dirname(__file__), "golden", "depth_mesh_error_golden.json")) as f:
        return json.load(f)["cases"]


DEPTH_MESH_CASES = _depth_mesh_golden()


@pytest.mark.parametrize("ci", range(len(DEPTH_MESH_CASES)))
def test_oracle_depth_mesh_matches_mpmath_golden(oracle, ci):
    """BracketedDepthMeshError (rig_calibrator.cc:641-673): the oracle against the
    50-digit mpmath restatement (tests/golden/make_golden_depth_mesh.py), rigid and
    affine depth_to_image, reference / interpolated frames, scale != 1. Residuals
    1e-12 relative, Jacobian 1e-8 of each block's largest entry; the numeric-diff
    mode (the reference's own Jacobian) within 1e-6 of it."""
    import numpy as np

    c = DEPTH_MESH_CASES[ci]
    blocks = [np.array(b) for b in c["blocks"]]
    rg = np.array(c["residual"])
    for mode, tol in ((oracle.ANALYTIC, 1e-8), (oracle.NUMDIFF, 1e-6)):
        r, J = oracle.depth_mesh_error(blocks, np.zeros(6, np.uint8), c["weight"], c["meas"], c["mesh"],
                                       *c["stamps"], mode=mode)
        assert np.abs(r - rg).max() <= 1e-12 * max(np.abs(rg).max(), 1.0)
        off = 0
        for b, blk in enumerate(blocks):
            n = 3 * blk.size
            Jg = np.array(c["jacobian"][b])
            scale = max(np.abs(Jg).max(), 1e-300)
            assert np.abs(J[off:off + n] - Jg).max() <= tol * scale, (mode, b)
            off += n


@pytest.mark.parametrize("models", [["radtan", "fov", "none"], ["rpc2", "radtan4", "rpc1"], ["rpc3", "none"]])
def test_faithful_numdiff_is_bit_identical(oracle, models):
    """Mode NUMDIFF_FAITHFUL (bench.py's cpu_baseline) keeps the reference's
    per-call work (CameraParameters deep copy + SetDistortion,
    rig_calibrator.cc:460-467; compute_rpc's validation, rpc_distortion.cc:116-124;
    Ceres' parameter copies and evaluation checks) around the same arithmetic:
    residuals and Jacobians equal mode NUMDIFF bit for bit, constant blocks
    included."""
    R = rig.make_rig(num_sensors=len(models), num_ref=10, num_points=120, obs_per_point=4, models=models, seed=17)
    P = rig.build_problem(R, rig.FloatFlags(camera_poses_to_float=()))
    r1, J1 = oracle.evaluate_mt(P, oracle.NUMDIFF, threads=2)
    r3, J3 = oracle.evaluate_mt(P, oracle.NUMDIFF_FAITHFUL, threads=2)
    assert np.array_equal(r1, r3) and np.array_equal(J1, J3)
