"""BracketedDepthError blocks (rig_calibrator.cc:522-609; config c5).

CPU: creation-time validation (the functor's block-size check, the image the
depth block belongs to) and the synthetic depth data at the true parameters.
GPU: residuals and Jacobian against the oracle restatement (exact derivative of
the same formulas, `oracle_depth_error`), rigid and affine depth_to_image,
with and without the Cauchy corrector, several constant-block patterns; the
normal equations including depth blocks against J^T r / J_b^T J_b built from the
oracle. Tolerances: residuals 1e-9 x max(|r|, 1), Jacobian 1e-9 of the block's
largest entry."""
import zlib

import numpy as np
import pytest

from multiview_amd import _lib, rig
from multiview_amd.evaluator import Evaluator, stats_labels
from oracle.normal_equations import normal_equations_reference


def _rig(affine=False, seed=3, **kw):
    return rig.make_rig(num_sensors=3, num_ref=10, num_points=120, obs_per_point=4, seed=seed,
                        depth_sensors=(2,), affine_depth=affine, **kw)


def _flags(affine=False, **kw):
    base = dict(depth_tri_weight=10.0, affine_depth_to_image=affine,
                depth_to_image_transforms_to_float=("cam2",), float_scale=True)
    base.update(kw)
    return rig.FloatFlags(**base)


def test_depth_data_at_truth():
    from oracle import oracle_py

    for affine in (False, True):
        R = _rig(affine)
        P = rig.build_problem(R, _flags(affine), use_init=False)
        assert P.num_depth_residuals == int((R.cam_type[R.obs_cid] == 2).sum())
        _, r, _ = oracle_py.evaluate_depth(P, oracle_py.RESIDUAL)
        assert np.abs(r).max() / 10.0 < 6 * 0.01  # weight 10, cloud noise sigma 1 cm


def _expect_status(P, status):
    from multiview_amd.evaluator import Evaluator

    with pytest.raises(_lib.MvbaError) as e:
        Evaluator(P)
    assert e.value.status == status, e.value


def test_depth_validation_before_device():
    """Checks that run in mvba_create before the device is touched (so they hold
    on CPU too): BracketedDepthError's block-size check (:534-543) and the image
    a depth block belongs to."""
    R = _rig()
    P = rig.build_problem(R, _flags())
    bad = P.depth_blocks.copy()
    bad[0, 4] = bad[0, 5]  # a 3-vector where the 1-element scale belongs
    P_bad = rig.build_problem(R, _flags())
    P_bad.depth_blocks = bad
    _expect_status(P_bad, _lib.MVBA_E_DEPTH_BLOCK_SIZES)
    P_orphan = rig.build_problem(R, _flags())
    P_orphan.depth_stamps = P_orphan.depth_stamps.copy()
    P_orphan.depth_stamps[0, 2] += 1e-3  # no image with these stamps
    _expect_status(P_orphan, _lib.MVBA_E_INVALID)


# ---------------------------------------------------------------- GPU parity
CASES = {
    "rigid": dict(affine=False, flags={}),
    "affine": dict(affine=True, flags={}),
    "rigid_const_dti": dict(affine=False, flags=dict(depth_to_image_transforms_to_float=(), float_scale=False)),
    "no_rig": dict(affine=False, flags=dict(no_rig=True, camera_poses_to_float=("ref_cam", "cam1", "cam2"))),
}


def _depth_close(got, ref):
    rg, Jg = got
    rr, Jr = ref
    assert np.abs(rg - rr).max() <= 1e-9 * max(np.abs(rr).max(), 1.0)
    for b in range(7):
        lo, hi = _lib.DJAC_BASE[b], (_lib.DJAC_BASE[b + 1] if b < 6 else _lib.DJAC_ROWS)
        scale = max(np.abs(Jr[:, lo:hi]).max(), 1e-300)
        assert np.abs(Jg[:, lo:hi] - Jr[:, lo:hi]).max() <= 1e-9 * scale, (b, np.abs(Jg[:, lo:hi] - Jr[:, lo:hi]).max())


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("apply_loss", [False, True])
def test_depth_eval_parity(oracle, name, apply_loss):
    c = CASES[name]
    R = _rig(c["affine"], seed=zlib.crc32(name.encode()) % 991)
    P = rig.build_problem(R, _flags(c["affine"], **c["flags"]))
    with Evaluator(P) as ev:
        ev.set_params()
        cost, r, J = ev.evaluate_depth(jacobian=True, apply_loss=apply_loss, robust_threshold=3.0)
    c_o, r_o, J_o = oracle.evaluate_depth(P, oracle.ANALYTIC, apply_loss=apply_loss, robust_threshold=3.0)
    assert np.isclose(cost, c_o, rtol=1e-11)
    _depth_close((r, J), (r_o, J_o))


def depth_normal_equations(P, layout, r, J):
    """J^T r and J_b^T J_b of the depth blocks in the mvba layouts (numpy)."""
    cam_g = np.zeros(layout["cam_grad_size"])
    cam_h = np.zeros(layout["cam_hess_size"])
    npts = layout["num_points"]
    pt_g = np.zeros((npts, 3))
    pt_h = np.zeros((npts, 6))
    cam_pos = {int(b): k for k, b in enumerate(layout["cam_block_ids"])}
    pt_pos = {int(b): k for k, b in enumerate(layout["point_block_ids"])}
    for j in range(P.num_depth_residuals):
        for b in range(7):
            bid = int(P.depth_blocks[j, b])
            if bid < 0:  # BracketedDepthMeshError: no point block
                continue
            size = int(P.block_size[bid])
            Jb = J[j, _lib.DJAC_BASE[b]:_lib.DJAC_BASE[b] + 3 * size].reshape(3, size)
            if b == 5:
                k = pt_pos.get(bid)
                if k is None:
                    continue
                H = Jb.T @ Jb
                pt_g[k] += Jb.T @ r[j]
                pt_h[k] += H[[0, 0, 0, 1, 1, 2], [0, 1, 2, 1, 2, 2]]
                continue
            k = cam_pos.get(bid)
            if k is None:
                continue
            go, ho = layout["cam_goff"][k], layout["cam_hoff"][k]
            cam_g[go:go + size] += Jb.T @ r[j]
            cam_h[ho:ho + size * size] += (Jb.T @ Jb).reshape(-1)
    return cam_g, cam_h, pt_g.reshape(-1), pt_h.reshape(-1)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["rigid", "affine"])
@pytest.mark.parametrize("apply_loss", [False, True])
def test_depth_linearize_parity(oracle, name, apply_loss):
    import torch

    c = CASES[name]
    R = _rig(c["affine"], seed=17)
    P = rig.build_problem(R, _flags(c["affine"], **c["flags"]))
    with Evaluator(P) as ev:
        ev.set_params()
        L = ev.lin_layout()
        cg = torch.zeros(L["cam_grad_size"], dtype=torch.float64, device="cuda")
        ch = torch.zeros(L["cam_hess_size"], dtype=torch.float64, device="cuda")
        pg = torch.zeros(3 * L["num_points"], dtype=torch.float64, device="cuda")
        ph = torch.zeros(6 * L["num_points"], dtype=torch.float64, device="cuda")
        cost = torch.zeros(1, dtype=torch.float64, device="cuda")
        ev.linearize_device(cg, ch, pg, ph, cost, apply_loss=apply_loss, robust_threshold=3.0)
        ev.sync()
    c_o, r_o, J_o = oracle.evaluate(P, oracle.ANALYTIC, apply_loss=apply_loss, robust_threshold=3.0)
    g, h, pgr, phr = normal_equations_reference(P, r_o, J_o, L)
    cd, rd, Jd = oracle.evaluate_depth(P, oracle.ANALYTIC, apply_loss=apply_loss, robust_threshold=3.0)
    g2, h2, pg2, ph2 = depth_normal_equations(P, L, rd, Jd)
    sizes = P.block_size[L["cam_block_ids"]]
    for got, ref, offs, ns in [(cg, g + g2, L["cam_goff"], sizes), (ch, h + h2, L["cam_hoff"], sizes * sizes)]:
        got = got.cpu().numpy()
        for o, n in zip(offs, ns):
            scale = max(np.abs(ref[o:o + n]).max(), 1e-300)
            assert np.abs(got[o:o + n] - ref[o:o + n]).max() <= 1e-9 * scale
    npt = L["num_points"]
    for got, ref, w in [(pg, pgr + pg2, 3), (ph, phr + ph2, 6)]:
        got = got.cpu().numpy().reshape(npt, w)
        ref = ref.reshape(npt, w)
        scale = np.maximum(np.abs(ref).max(axis=1, keepdims=True), 1e-300)
        assert (np.abs(got - ref) <= 1e-9 * scale).all()
    assert np.isclose(cost.item(), c_o + cd, rtol=1e-11)


@pytest.mark.gpu
def test_residual_stats_match_oracle(oracle):
    """mvba_residual_stats = evalResiduals + calc_residuals_stats: raw residuals
    divided by their scale, grouped by name, percentiles by index; against the
    oracle's residuals fed to the oracle's restatement of calc_residuals_stats.
    Pixel, depth (scale depth_tri_weight) and XYZ prior (scale tri_weight) groups."""
    R = _rig(False, seed=23)
    P = rig.build_problem(R, _flags(False, tri_weight=0.5, tri_robust_threshold=0.1))
    P.params = P.params.copy()
    P.params[P.block_offset[P.xyz_block]] += np.linspace(-0.05, 0.05, P.num_xyz_residuals)
    names = R.sensor_names
    with Evaluator(P) as ev:
        ev.set_params()
        rows = ev.residual_stats(names)
    _, r, _ = oracle.evaluate(P, oracle.RESIDUAL)
    _, rd, _ = oracle.evaluate_depth(P, oracle.RESIDUAL)
    _, rx, _ = oracle.evaluate_xyz(P)
    ncam = len(P.camera_dist_size)
    vals = np.concatenate([r.reshape(-1), (rd / P.depth_weight[:, None]).reshape(-1),
                           (rx.reshape(-1, 3) / P.xyz_weight[:, None]).reshape(-1)])
    ids = np.concatenate([(2 * P.residual_camera[:, None] + np.arange(2)).reshape(-1),
                          (2 * ncam + np.tile(np.arange(3), rd.shape[0])),
                          (2 * ncam + 3 + np.tile(np.arange(3), P.num_xyz_residuals))]).astype(np.int32)
    ng = 2 * ncam + 12
    ref, counts = oracle.residual_stats(vals, ids, ng)
    labels = stats_labels(names)
    expect = sorted([(labels[g], *ref[g], int(counts[g])) for g in range(ng) if counts[g] > 0],
                    key=lambda t: t[0])
    assert [e[0] for e in expect] == [g[0] for g in rows]
    assert "tri_x_m" in [g[0] for g in rows]
    for g, e in zip(rows, expect):
        assert g[5] == e[5]
        assert np.allclose(g[1:5], e[1:5], rtol=1e-9, atol=1e-12), (g, e)
    text = Evaluator.format_residual_stats(rows, "before opt")
    assert text.splitlines()[0] == "The 25, 50, 75, and 100th percentile residual stats before opt"
