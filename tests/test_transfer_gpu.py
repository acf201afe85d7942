"""Host hand-over of evaluations (mvba_transfer.hip, mvba_transfer_host.cpp):
the device rewrites the column planes into AddResidualBlock-order rows and one
device-to-host copy moves them (the layout Ceres' CostFunction::Evaluate fills,
rig_calibrator.cc:1695-1699).

Checked against an independent host transposition of the device planes
(evaluate_device + the slot order, numpy), which the parity tests pin to the
oracle: full layout (mvba_evaluate), packed layout for several transfer sets
(mvba_evaluate_packed), Cauchy corrector, pinned and pageable destinations, and
a copy larger than the two 32 MB staging buffers."""
import numpy as np
import pytest
import torch

from multiview_amd import _lib, rig
from multiview_amd.evaluator import Evaluator, PinnedBuffer

pytestmark = pytest.mark.gpu

JAC_BASE = np.array(_lib.JAC_BASE)


def _planes_to_rows(ev, P, loss, thr=3.0):
    """Independent restatement: device planes -> insertion-order rows (numpy)."""
    v = ev.device_view()
    ld, rows = int(v.ld), int(v.jac_rows)
    res = torch.empty((2, ld), dtype=torch.float64, device="cuda")
    jac = torch.empty((rows, ld), dtype=torch.float64, device="cuda")
    ev.evaluate_device(jacobian=True, residuals=res, jac=jac, ld=ld)
    ev.sync()
    order = ev.order()
    live = order >= 0
    r = res.cpu().numpy()[:, :order.size][:, live].T
    J = jac.cpu().numpy()[:, :order.size][:, live].T
    idx = order[live]
    n = P.num_residuals
    R = np.empty((n, 2))
    JJ = np.zeros((n, rows))
    R[idx] = r
    JJ[idx] = J
    # constant blocks / unused distortion rows are not written by K1: zero them
    K = P.camera_dist_size[P.residual_camera]
    for i_b, (lo, w) in enumerate(zip(JAC_BASE, (7, 7, 7, 3, 1, 1, 2, None))):
        const = P.block_constant[P.residual_blocks[:, i_b]].astype(bool)
        hi = lo + 2 * w if w is not None else rows
        JJ[const, lo:hi] = 0.0
    col = np.arange(rows)[None, :]
    JJ[(col >= 56 + 2 * K[:, None])] = 0.0
    sr = np.ones(n)
    if loss:
        s2 = (R ** 2).sum(1)
        c = 1.0 / (thr * thr)
        sr = np.sqrt(np.maximum(np.finfo(float).tiny, 1.0 / (1.0 + s2 * c)))
    return R * sr[:, None], JJ * sr[:, None]


def _pack(P, J, transfer, off):
    """Packed rows from full rows, per mvba_set_transfer_blocks' layout: residual
    i's transferred blocks in block order at off[i] (rows in device order)."""
    K = P.camera_dist_size[P.residual_camera]
    out = np.full(int(off[-1]), np.nan)
    for i in range(P.num_residuals):
        row = [J[i, JAC_BASE[b]:JAC_BASE[b] + 2 * (K[i] if b == 7 else _lib.FIXED_BLOCK_SIZES[b])]
               for b in range(8) if transfer[P.residual_blocks[i, b]]]
        if row:
            row = np.concatenate(row)
            out[off[i]:off[i] + row.size] = row
    assert not np.isnan(out).any()  # the rows tile the packed buffer
    return out


@pytest.fixture(scope="module")
def problem():
    R = rig.make_rig(num_sensors=3, num_ref=10, num_points=300, obs_per_point=5,
                     models=["radtan", "rpc2", "fov"], seed=7)
    return rig.build_problem(R)


@pytest.mark.parametrize("loss", [False, True])
def test_full_rows_match_planes(problem, loss):
    P = problem
    with Evaluator(P) as ev:
        ev.set_params()
        r_ref, J_ref = _planes_to_rows(ev, P, loss)
        cost, r, J = ev.evaluate(jacobian=True, apply_loss=loss)
    assert np.array_equal(r, r_ref)
    assert np.array_equal(J, J_ref)
    if not loss:
        assert cost == pytest.approx(0.5 * (r_ref ** 2).sum(), rel=1e-12)


@pytest.mark.parametrize("pattern", ["default", "all", "poses_only", "none", "random"])
def test_packed_rows(problem, pattern):
    P = problem
    nb = len(P.block_size)
    rng = np.random.default_rng(3)
    transfer = {
        "default": None,
        "all": np.ones(nb, np.uint8),
        "poses_only": (P.block_size == 7).astype(np.uint8),
        "none": np.zeros(nb, np.uint8),
        "random": (rng.random(nb) < 0.5).astype(np.uint8),
    }[pattern]
    with Evaluator(P) as ev:
        ev.set_params()
        r_ref, J_ref = _planes_to_rows(ev, P, True)
        off = ev.set_transfer_blocks(transfer)
        t = (1 - P.block_constant).astype(np.uint8) if transfer is None else transfer
        expect = _pack(P, J_ref, t, off)
        with PinnedBuffer(max(expect.size, 1)) as buf:
            _, r, Jp = ev.evaluate_packed(jacobian=True, apply_loss=True, out=buf.array)
            assert np.array_equal(r, r_ref)
            assert np.array_equal(Jp[:expect.size], expect)
        _, r2, Jp2 = ev.evaluate_packed(jacobian=True, apply_loss=True)  # pageable destination
        assert np.array_equal(Jp2, expect) and np.array_equal(r2, r_ref)
        # residual-only pass leaves the packed layout alone
        _, r3, none = ev.evaluate_packed(jacobian=False, apply_loss=True)
        assert none is None and np.array_equal(r3, r_ref)


def test_large_copy_through_staging():
    """> 64 MB of rows: several chunks through the two pinned staging buffers."""
    R = rig.make_rig(num_sensors=3, num_ref=60, num_points=40000, obs_per_point=5,
                     models=["radtan", "radtan", "radtan"], seed=11)
    P = rig.build_problem(R)
    P.block_constant[:] = 0
    with Evaluator(P) as ev:
        ev.set_params()
        assert P.num_residuals * ev.stride * 8 > 64 << 20
        r_ref, J_ref = _planes_to_rows(ev, P, False)
        _, r, J = ev.evaluate(jacobian=True)
        assert np.array_equal(r, r_ref) and np.array_equal(J, J_ref)
        with PinnedBuffer(P.num_residuals * ev.stride) as buf:
            off = ev.set_transfer_blocks(np.ones(len(P.block_size), np.uint8))
            _, r2, Jp = ev.evaluate_packed(jacobian=True, out=buf.array)
            assert off[-1] == J_ref.size  # one distortion size everywhere: packed == full rows
            rows = Jp[off[:-1, None] + np.arange(ev.stride)[None, :]]
            assert np.array_equal(rows, J_ref)
